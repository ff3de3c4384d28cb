// tv.hip -- threshold-v on gfx950.
//
// Reference: ThresholdvCompressor::impl_naive (the path actually compiled under
// -march=broadwell: thresholdv.cpp:137-139, 292-293 -> 40-83), first threshold
// impl_get_first_threshold (:27-37).
//
// Semantics: per element, |x| >= t is emitted in index order
// while fewer than `cap` were found (idx = i, idx_offset ignored); every
// qualifier is counted; gmax = max |x|.  AIMD: k > cnt -> t *= 0.99 (double);
// k < cnt -> t = fma(0.01*cnt/k, gmax, t) in double (GCC contracts it at -O3).
// Returns min(cnt, cap).  The state is keyed by the src pointer (:44).
//
// GPU structure: two launches (tv_chunk, tv_fold), no waits.  tv_chunk: one
// 256-thread workgroup per 32 KiB chunk (tile.h's tile; the hardware hands
// chunks to whichever CU frees a slot first, so no CU's share sets the end):
// every lane's 8 float4 loads in flight at once, the chunk's qualifier count,
// max |x| and its first TV_CAPC qualifiers (position, bits) in position order
// into the chunk's list.  tv_fold: each workgroup sums the counts of the
// chunks before its TV_CPW chunks, one wave per chunk copies the list to its
// offset (capped; a chunk with more qualifiers than its list holds is read
// again in position order), and the last workgroup folds every count and
// maximum into the AIMD threshold and the count.  One read of the bucket.
//
// Before (STG_TV_PASS=1, kept for A/B): one launch, HBM-bound (tv_pass).  1024-thread workgroups
// (STG_TV_WPC per CU) take contiguous ranges of the bucket in ticket order; 16 waves
// stream the range with a rolling pipeline of SCAN_D nontemporal float4 loads
// per lane, count the qualifiers and max|x|, and list the qualifiers
// (position, value) in LDS; the range publishes its count, sums the counts of
// the earlier ranges (look-back: taken earlier, so their workgroups are
// running or done; no co-residency needed) and writes its list in position
// order at that offset
// (capped).  A range whose list overflowed its LDS capacity is re-scanned in
// order.  The last range folds the counts and maxima into the AIMD threshold
// and the count.
#include <algorithm>
#include <cstdlib>

#include "tile.h"
#include "ws.h"

namespace stg {

namespace {

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

#ifndef STG_TV_TWG
#define STG_TV_TWG 1024
#endif
constexpr uint32_t TWG = STG_TV_TWG;  // threads per workgroup (16 waves)
constexpr uint32_t TNW = TWG / 64;
#ifndef STG_TV_WPC
#define STG_TV_WPC 1  // workgroups per CU (1 with 6 loads in flight per lane: 52.3 us at C3; 2 with 4: 55.6)
#endif
#ifndef STG_TV_SCAN_D
#define STG_TV_SCAN_D 6
#endif
constexpr uint32_t SCAN_D = STG_TV_SCAN_D;  // float4 loads in flight per lane
constexpr uint32_t LCAP = TV_SCAP * TWG / 1024u;  // qualifiers listed in LDS per range

__global__ void tv_init_state(KeyState *st, const RSel *rs) {
    st->t = u2f(rs->prefix);
    st->inc = 0.f;
    st->init = 1;
}

// Range of workgroup w in float4 units; the ragged n % 4 tail belongs to the
// last range.  (Ranges tapered over the tickets, so that later tickets get
// less, measured 3-7 % slower at C3.)
struct TvRange {
    uint64_t lo, len;
};
__device__ __forceinline__ TvRange tv_range(uint64_t n4, uint32_t G, uint32_t w) {
    const uint64_t per = n4 / G, rem = n4 % G;
    TvRange r;
    r.lo = w * per + std::min<uint64_t>(w, rem);
    r.len = per + (w < rem ? 1u : 0u);
    return r;
}

struct TvArgs {
    const float *src;
    uint64_t n;
    uint32_t k, cap;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    uint64_t *desc;      // per range: {call tag:32 | qualifier count:32}
    uint64_t *rmax;      // per range: {call tag:32 | max |x| bits:32}
    uint32_t tag;        // this call's tag, >= 1
    uint64_t *ticket;    // ranges taken: monotonic over the workspace's calls (zero at creation)
    uint64_t base;       // its value when this call starts (G per earlier call)
    uint32_t *fail;      // the workspace's sticky failure word
    uint32_t *dbg;       // diagnostics (STG_TV_STAMPS builds): phase stamps at words 40..49
    uint32_t withhold;   // tests (STG_DEBUG_TV_WITHHOLD=1): range 0 never publishes its count, so every
                         // later range's look-back runs out its bound: the failure path end to end
};

#ifndef STG_TV_STAMPS
#define STG_TV_STAMPS 0
#endif
// s_memrealtime (100 MHz) phase stamps: the maximum over the ranges by
// atomicMax, or one range's by a plain store
#define TV_STAMP_MAX(w)                                                                              \
    do {                                                                                             \
        if (STG_TV_STAMPS && threadIdx.x == 0) atomicMax(&a.dbg[w], (uint32_t)__builtin_amdgcn_s_memrealtime()); \
    } while (0)
#define TV_STAMP_IF(cond, w)                                                                         \
    do {                                                                                             \
        if (STG_TV_STAMPS && threadIdx.x == 0 && (cond)) a.dbg[w] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)

// One launch: the workgroup with ticket r streams range r, publishes its count,
// sums the counts of the earlier ranges (look-back) and writes the range's
// qualifiers at that offset in position order; range G-1 folds the counts and
// maxima into the AIMD threshold and the count.
__global__ void __launch_bounds__(TWG, 8) tv_pass(TvArgs a) {
    __shared__ uint32_t s_pos[LCAP];
    __shared__ float s_val[LCAP];
    __shared__ uint32_t s_n, s_r, s_cnt[TNW], s_max[TNW];
    __shared__ uint64_t s_P, s_psum[TNW];
    __shared__ uint32_t sh[TNW + 1];
    const uint32_t G = gridDim.x, tid = threadIdx.x;
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    uint32_t t_start = 0;
    if (STG_TV_STAMPS && tid == 0) t_start = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        s_n = 0;
        s_r = (uint32_t)(g_add(a.ticket, 1ull) - a.base);
    }
    // read before this range's count is published: the last workgroup
    // rewrites the state only after every range's count is in
    const float t = a.state->t;
    __syncthreads();
    const uint32_t r = s_r;  // ranges in ticket order
    if (STG_TV_STAMPS && tid == 0) {
        if (r == 0) a.dbg[40] = t_start;
        atomicMax(&a.dbg[41], t_start);
    }
    TV_STAMP_MAX(42);  // ticket in
    uint32_t s_tkt_time = 0;
    if (STG_TV_STAMPS && tid == 0) s_tkt_time = (uint32_t)__builtin_amdgcn_s_memrealtime();
    const uint64_t n = a.n, n4 = n / 4;
    const TvRange R = tv_range(n4, G, r);
    // the range as a bounded buffer: lanes past it read zeros (launch_tv keeps
    // every range below 2^28 float4)
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(a.src + R.lo * 4), 0, (uint32_t)(R.len * 16), 0x00020000);
    const uint32_t steps = (uint32_t)((R.len + 63) / 64);  // 64 float4 per wave step
    const uint32_t mine = steps > wave ? (steps - wave + TNW - 1) / TNW : 0u;
    auto load = [&](uint32_t m) -> float4 {
        uint32_t voff = (wave * 64 + lane) * 16u;
        asm volatile("" : "+v"(voff));
        const u4v q = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + m * (TNW * 1024u), 0, 2 /* nt */);
        return make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w));
    };
    uint32_t cnt = 0, mx = 0;
    float4 v[SCAN_D];
#pragma unroll
    for (uint32_t u = 0; u < SCAN_D; ++u) v[u] = load(u);
    for (uint32_t m0 = 0; m0 < mine; m0 += SCAN_D) {
#pragma unroll
        for (uint32_t u = 0; u < SCAN_D; ++u) {
            // consume the slot before loading into it (loading first made the
            // compiler move registers at the back-edge behind a wait for every load)
            const float4 x = v[u];
            const uint32_t f = ((m0 + u) * TNW + wave) * 64 + lane;  // float4 within the range
            const bool in = f < R.len;
            const float a0 = fabsf(x.x), a1 = fabsf(x.y), a2 = fabsf(x.z), a3 = fabsf(x.w);
            if (in) mx = max(mx, max(max(f2u(a0), f2u(a1)), max(f2u(a2), f2u(a3))));
            const uint32_t q = in ? ((uint32_t)(a0 >= t) | ((uint32_t)(a1 >= t) << 1) | ((uint32_t)(a2 >= t) << 2) |
                                     ((uint32_t)(a3 >= t) << 3))
                                  : 0u;
            if (__ballot(q != 0) && q) {  // rare: list this lane's qualifiers
                const uint32_t c = (uint32_t)__popc(q);
                cnt += c;
                uint32_t o = atomicAdd(&s_n, c);
                const uint32_t p0 = (uint32_t)((R.lo + f) * 4);
                const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if ((q >> j) & 1u) {
                        if (o < LCAP) { s_pos[o] = p0 + j; s_val[o] = xs[j]; }
                        ++o;
                    }
                }
            }
            v[u] = load(m0 + u + SCAN_D);
        }
    }
    // the ragged tail (n % 4 elements) closes the last range
    if (r == G - 1 && tid == 0) {
        for (uint64_t e = n4 * 4; e < n; ++e) {
            const float x = a.src[e], ax = fabsf(x);
            mx = max(mx, f2u(ax));
            if (ax >= t) {
                const uint32_t o = atomicAdd(&s_n, 1u);
                ++cnt;
                if (o < LCAP) { s_pos[o] = (uint32_t)e; s_val[o] = x; }
            }
        }
    }
    cnt = wave_sum(cnt);
    mx = wave_max(mx);
    if (lane == 0) { s_cnt[wave] = cnt; s_max[wave] = mx; }
    __syncthreads();
    TV_STAMP_MAX(44);  // streaming done
    if (STG_TV_STAMPS && tid == 0 && a.cap >= 4 * G) {  // per range, at the end of idx: block, start, ticket in, stream end
        uint32_t *o = a.idx + a.cap - 4 * G + 4 * r;
        o[0] = blockIdx.x;
        o[1] = t_start;
        o[2] = s_tkt_time;
        o[3] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    }
    TV_STAMP_IF(r == 0, 43);
    TV_STAMP_IF(r == G - 1, 47);
    const uint32_t listed = s_n;
    uint32_t c = 0;
    for (uint32_t i = 0; i < TNW; ++i) c += s_cnt[i];
    if (tid == 0) {  // publish: the tagged maximum and the tagged count (no order between them)
        uint32_t m = 0;
        for (uint32_t i = 0; i < TNW; ++i) m = max(m, s_max[i]);
        st_sc1(&a.rmax[r], ((uint64_t)a.tag << 32) | m);
        if (!(a.withhold && r == 0)) st_sc1(&a.desc[r], ((uint64_t)a.tag << 32) | c);
    }
    // look-back: the counts of ranges 0 .. r-1 (taken earlier, so held by
    // running or finished workgroups), one per thread in one round trip;
    // stale ones are polled by their lane with s_sleep (a few lanes at most:
    // the ranges finish streaming together)
    uint64_t Pl = 0;
    bool gave_up = false;
    constexpr uint32_t LB = (TV_MAXG + TWG - 1) / TWG;  // earlier ranges per thread, all loaded at once
    uint64_t dl[LB];
#pragma unroll
    for (uint32_t q = 0; q < LB; ++q) {
        const uint32_t i = tid + q * TWG;
        dl[q] = i < r ? ld_sc1(&a.desc[i]) : (uint64_t)a.tag << 32;
    }
#pragma unroll
    for (uint32_t q = 0; q < LB; ++q) {
        const uint32_t i = tid + q * TWG;
        uint64_t d = dl[q], st = 0;
        for (uint32_t spins = 0; (uint32_t)(d >> 32) != a.tag; ++spins) {
            __builtin_amdgcn_s_sleep(8);
            d = ld_sc1(&a.desc[i]);
            if (spin_expired(spins, st)) { gave_up = true; break; }  // 200 ms: the count is poisoned below
        }
        Pl += (uint32_t)d;
    }
    if (gave_up) g_or(a.fail, FAIL_SPIN_TIMEOUT);
    Pl = wave_sum64(Pl);
    if (lane == 0) s_psum[wave] = Pl;
    __syncthreads();
    if (tid == 0) {
        uint64_t t2 = 0;
        for (uint32_t i = 0; i < TNW; ++i) t2 += s_psum[i];
        s_P = t2;
    }
    __syncthreads();
    const uint64_t P = s_P;
    const uint32_t cap_e = STG_TV_STAMPS && a.cap >= 4 * G ? a.cap - 4 * G : a.cap;  // stamps build: keep the tail
    TV_STAMP_MAX(45);  // look-back done
    TV_STAMP_IF(r == G - 1, 48);
    if (P < cap_e && c) {
        const uint32_t m = (uint32_t)std::min<uint64_t>(c, cap_e - P);
        if (listed <= LCAP) {
            // position order: rank = listed entries with a smaller position
            for (uint32_t e = tid; e < listed; e += TWG) {
                const uint32_t p = s_pos[e];
                uint32_t rk = 0;
                for (uint32_t x = 0; x < listed; ++x) rk += s_pos[x] < p;
                if (rk < m) {
                    a.idx[P + rk] = p;
                    a.val[P + rk] = s_val[e];
                }
            }
        } else {
            // the range's list overflowed: its qualifiers again, in order
            const uint64_t units = R.len + (r == G - 1 && n % 4 ? 1u : 0u);  // + the ragged tail
            uint64_t base = 0;
            for (uint64_t f0 = 0; f0 < units && base < m; f0 += TWG) {
                const uint64_t f = f0 + tid;
                uint32_t q = 0;
                float xs[4] = {0.f, 0.f, 0.f, 0.f};
                if (f < units) {
#pragma unroll
                    for (uint32_t j = 0; j < 4; ++j) {
                        const uint64_t e = (R.lo + f) * 4 + j;
                        if (e < n) {
                            xs[j] = a.src[e];
                            q |= (uint32_t)(fabsf(xs[j]) >= t) << j;
                        }
                    }
                }
                uint32_t total;
                const uint32_t ex = blk_excl_scan<TNW>((uint32_t)__popc(q), sh, &total);
                uint64_t o = base + ex;
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) {
                    if ((q >> j) & 1u) {
                        if (o < m) {
                            a.idx[P + o] = (uint32_t)((R.lo + f) * 4 + j);
                            a.val[P + o] = xs[j];
                        }
                        ++o;
                    }
                }
                base += total;
            }
        }
    }
    TV_STAMP_MAX(49);  // emission issued
    // the last range has seen every range's count (the look-back), and each
    // range stored its maximum before its count: fold them
    if (r != G - 1) return;
    uint32_t gm = 0;
    for (uint32_t i = tid; i < G; i += TWG) {  // every range's tagged maximum
        uint64_t x = ld_sc1(&a.rmax[i]);
        uint64_t st = 0;
        for (uint32_t spins = 0; (uint32_t)(x >> 32) != a.tag; ++spins) {
            __builtin_amdgcn_s_sleep(8);
            x = ld_sc1(&a.rmax[i]);
            if (spin_expired(spins, st)) { g_or(a.fail, FAIL_SPIN_TIMEOUT); break; }
        }
        gm = max(gm, (uint32_t)x);
    }
    const uint64_t cntall = P + c;
    gm = wave_max(gm);
    if (lane == 0) s_max[wave] = gm;
    __syncthreads();
    if (tid == 0) {
        uint32_t g = 0;
        for (uint32_t i = 0; i < TNW; ++i) g = max(g, s_max[i]);
        const float gmax = n ? u2f(g) : -1.f;
        float nt = t;
        if ((uint64_t)a.k > cntall) nt = (float)((double)t * 0.99);
        else if ((uint64_t)a.k < cntall) nt = (float)fma(0.01 * (double)cntall / (double)a.k, (double)gmax, (double)t);
        a.state->t = nt;
        a.state->init = 1;
        *a.count_out = (uint32_t)std::min<uint64_t>(cntall, a.cap);
        if (ld_sc1(a.fail)) *a.count_out = POISON_COUNT;  // a bounded wait gave up: untrusted output
    }
    TV_STAMP_IF(true, 46);  // the fold written
}

hipError_t launch_tv_pass(const TvLaunch &a, const DevWS &ws, hipStream_t s) {
    // STG_TV_WPC workgroups per CU, each with >= 64 KiB of the bucket
    const uint64_t n4 = a.n / 4;
    const uint32_t G = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(std::min<uint64_t>((uint64_t)STG_TV_WPC * a.num_cu, TV_MAXG), (n4 + 4095) / 4096));
    if (n4 / G + 1 >= (1ull << 28)) return hipErrorInvalidValue;  // a range must fit one buffer descriptor
    TvArgs f;
    f.src = a.src;
    f.n = a.n;
    f.k = a.k;
    f.cap = a.cap;
    f.idx = a.idx;
    f.val = a.val;
    f.count_out = a.count_out;
    f.state = a.state;
    f.desc = reinterpret_cast<uint64_t *>(ws.tile_cnt);
    f.rmax = reinterpret_cast<uint64_t *>(ws.tile_aux);
    f.tag = a.tag;
    f.fail = ws.fail;
    f.dbg = ws.misc;
    f.ticket = ws.tv_ticket;
    f.base = a.ticket_base;
    static const bool withhold = getenv("STG_DEBUG_TV_WITHHOLD") && atoi(getenv("STG_DEBUG_TV_WITHHOLD")) == 1;
    f.withhold = withhold && G > 1;
    if (a.grid_out) *a.grid_out = G;
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    tv_pass<<<G, TWG, 0, s>>>(f);
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}


// ---------------------------------------------------------------------------
// static chunks: tv_chunk, then tv_fold
// ---------------------------------------------------------------------------
constexpr uint32_t TV_CH = 2048;    // elements per chunk: one wave's 64 lanes x 8 float4 (8 KiB)
constexpr uint32_t TV_CAPC = 32;    // qualifiers listed per chunk
constexpr uint32_t TV_CPW = 128;    // chunks per tv_fold workgroup (a group)
constexpr uint32_t TV_FR = TV_CPW * TV_CAPC / STG_WG;  // list entries per tv_fold thread
static_assert(TV_CPW * TV_CAPC % STG_WG == 0 && TV_CPW <= STG_WG, "fold shape");

struct TvcArgs {
    const float *src;
    uint64_t n;
    uint32_t nc, ng, k, cap;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    uint2 *lst;            // chunk c's list: lst[c TV_CAPC ..], {position, bits}
    uint32_t *cnt;         // chunk c's qualifier count
    uint32_t *gsum, *gmax;  // this call's parity: per group of TV_CPW chunks, the counts' sum and max |x| bits
    uint32_t *zsum, *zmax;  // the other parity's, zeroed here for the next call
    uint32_t zng;          // ... over the groups its last call used
    float *tcall;          // this call's threshold, for tv_fold (whose last workgroup rewrites the state)
    uint32_t *fail;
};

#ifndef STG_TV_WPE
#define STG_TV_WPE 4  // tv_chunk waves per SIMD (two chunks' data in registers: <= 128 VGPRs); workgroups per CU
#endif
// Every wave scans its own static range of 8 KiB chunks with no barrier and
// no LDS: each lane's eight nontemporal float4 loads of a chunk in flight,
// the chunk's qualifiers ranked by ballots (position order is (u, lane, j))
// and listed straight to global memory, its count stored and added to its
// group's sum.  Waves stream independently, as a plain read does: 6.6 TB/s
// on 256 MiB (tools/ubench_stream.hip); one workgroup per 32 KiB chunk with
// a cross-wave ordering (two barriers a chunk) read 4.4 TB/s here.
template <bool VEC>
__global__ void __launch_bounds__(STG_WG) __attribute__((amdgpu_waves_per_eu(STG_TV_WPE, 8))) tv_chunk(const TvcArgs a) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t gw = blockIdx.x * STG_WAVES + wave, nw = gridDim.x * STG_WAVES;
    const uint32_t per = a.nc / nw, rem = a.nc % nw;
    const uint32_t c_lo = gw * per + std::min(gw, rem), c_hi = c_lo + per + (gw < rem ? 1u : 0u);
    const uint32_t n32 = (uint32_t)a.n;  // (launch_tv refuses n >= 2^32)
    const float t = a.state->t;
    if (blockIdx.x == 0 && threadIdx.x == 0) *a.tcall = t;
    const uint64_t lt = lane ? ~0ull >> (64 - lane) : 0ull;
    uint32_t mx = 0;  // this lane's max |x| bits over the wave's chunks
    auto chunk = [&](uint32_t c, const float4 (&v)[TILE_U], bool full) __attribute__((always_inline)) {
        const uint32_t base = c * TV_CH;
        uint2 *const dst = a.lst + (size_t)c * TV_CAPC;
        uint32_t wloc = 0;  // (uniform)
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) {
            const uint32_t e = base + 4 * (u * 64 + lane);
            uint32_t qn = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // (selects, no branches)
                const float ax = fabsf(comp(v[u], j));
                const bool in = full || e + j < n32;
                mx = in ? max(mx, f2u(ax)) : mx;
                qn |= (in && ax >= t) ? 1u << j : 0u;
            }
            uint32_t below = 0, wt = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint64_t bj = __ballot((qn >> j) & 1u);
                below += (uint32_t)__popcll(bj & lt);
                wt += (uint32_t)__popcll(bj);
            }
            if (qn) {
                uint32_t r = wloc + below;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if ((qn >> j) & 1u) {
                        if (r < TV_CAPC) dst[r] = make_uint2(e + j, f2u(comp(v[u], j)));
                        ++r;
                    }
            }
            wloc += wt;
        }
        if (lane == 0) {
            a.cnt[c] = wloc;
            // the group's sum: no return
            if (wloc) __hip_atomic_fetch_add(gp(&a.gsum[c / TV_CPW]), wloc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    };
    const uint32_t c_full = VEC ? std::min<uint32_t>(c_hi, n32 / TV_CH) : c_lo;
    // whole chunks: nontemporal buffer loads (read once), the next chunk's
    // issued before this one's stores -- gfx950 counts stores and loads in one
    // in-order vmcnt, so a load issued after a store waits for the store too
    auto load = [&](uint32_t c, float4 (&v)[TILE_U]) __attribute__((always_inline)) {
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.src + (size_t)c * TV_CH), 0, TV_CH * 4u, 0x00020000);
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) {  // (u's offset as the scalar offset)
            const u4v q = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 16u, u * 1024u, 2 /* nt */);
            v[u] = make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), __uint_as_float(q.w));
        }
    };
    uint32_t c = c_lo;
    if (c < c_full) {
        float4 v[TILE_U], vn[TILE_U];
        load(c, v);
        for (; c < c_full; ++c) {
            if (c + 1 < c_full) load(c + 1, vn);
            chunk(c, v, true);
#pragma unroll
            for (uint32_t u = 0; u < TILE_U; ++u) v[u] = vn[u];
        }
    }
    for (; c < c_hi; ++c) {  // the partial last chunk, or an unaligned bucket: guarded loads
        float4 v[TILE_U];
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) {
            const uint32_t e = c * TV_CH + 4 * (u * 64 + lane);
            float x[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = e + j < n32 ? a.src[e + j] : 0.f;
            v[u] = make_float4(x[0], x[1], x[2], x[3]);
        }
        chunk(c, v, false);
    }
    // the wave's maximum into its first chunk's group (the fold takes the
    // maximum over every group)
    mx = wave_max(mx);
    if (lane == 0 && c_lo < c_hi)
        __hip_atomic_fetch_max(gp(&a.gmax[c_lo / TV_CPW]), mx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Chunk c's qualifiers again, in position order, by one wave: the first m
// at out offset `off` (a chunk whose list overflowed).
// (plain arguments: a reference to the kernel's argument block would put the
// whole block in scratch)
__device__ __noinline__ void tv_rescan(const float *src, uint64_t n, uint32_t *idx, float *val, uint32_t c,
                                       uint64_t off, uint32_t m, float t) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t lt = lane ? ~0ull >> (64 - lane) : 0ull;
    const size_t base = (size_t)c * TV_CH, end = std::min<size_t>(base + TV_CH, n);
    uint32_t done = 0;
    for (size_t e0 = base; e0 < end && done < m; e0 += 256) {  // 64 lanes x 4 elements
        const size_t e = e0 + 4 * lane;
        float x[4];
        uint32_t q = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            x[j] = e + j < end ? src[e + j] : 0.f;
            if (e + j < end && fabsf(x[j]) >= t) q |= 1u << j;
        }
        uint32_t r = done, tot = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint64_t b = __ballot((q >> j) & 1u);
            r += (uint32_t)__popcll(b & lt);
            tot += (uint32_t)__popcll(b);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if ((q >> j) & 1u) {
                if (r < m) {
                    idx[off + r] = (uint32_t)(e + j);
                    val[off + r] = x[j];
                }
                ++r;
            }
        done += tot;
    }
}

// Group g (chunks [32 g, 32 g + 32)): the sums of the groups before it, its
// chunks' counts, then their lists -- three round trips -- and the copy.  The
// last group also folds every group's sum and maximum into the AIMD state.
__global__ void __launch_bounds__(STG_WG) tv_fold(const TvcArgs a) {
    __shared__ uint32_t sh[STG_WAVES + 1], s_cnt[TV_CPW], s_off[TV_CPW];
    __shared__ uint64_t sh64[STG_WAVES];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6, g = blockIdx.x, nc = a.nc;
    const uint32_t c0 = g * TV_CPW, nown = std::min(TV_CPW, nc - c0);
    const bool last = g + 1 == gridDim.x;
    if (g == 0)  // the next call's parity (this call never touches it)
        for (uint32_t i = tid; i < a.zng; i += STG_WG) { a.zsum[i] = 0u; a.zmax[i] = 0u; }
    const uint32_t own = tid < nown ? a.cnt[c0 + tid] : 0u;
    uint64_t before = 0, all = 0;
    uint32_t gm = 0;
    const uint32_t lim = last ? a.ng : g;
    for (uint32_t i = tid; i < lim; i += STG_WG) {
        const uint32_t x = a.gsum[i];
        if (i < g) before += x;
        all += x;
        if (last) gm = max(gm, a.gmax[i]);
    }
    {
        uint32_t tot;
        const uint32_t ex = blk_excl_scan<STG_WAVES>(own, sh, &tot);
        if (tid < TV_CPW) { s_cnt[tid] = own; s_off[tid] = ex; }
    }
    before = blk_sum64<STG_WAVES>(before, sh64);  // (its barriers also publish s_cnt / s_off)
    // the lists: entry p = tid + 256 r is chunk p / 64's slot p % 64
    uint2 e[TV_FR];
#pragma unroll
    for (uint32_t r = 0; r < TV_FR; ++r) {
        const uint32_t p = tid + STG_WG * r, i = p / TV_CAPC, l = p % TV_CAPC;
        e[r] = i < nown && l < min(s_cnt[i], TV_CAPC) ? a.lst[(size_t)(c0 + i) * TV_CAPC + l] : make_uint2(0u, 0u);
    }
#pragma unroll
    for (uint32_t r = 0; r < TV_FR; ++r) {
        const uint32_t p = tid + STG_WG * r, i = p / TV_CAPC, l = p % TV_CAPC;
        if (i < nown && s_cnt[i] <= TV_CAPC && l < s_cnt[i]) {
            const uint64_t o = before + s_off[i] + l;
            if (o < a.cap) {
                a.idx[o] = e[r].x;
                a.val[o] = u2f(e[r].y);
            }
        }
    }
    // (not the state: the last group rewrites it, maybe before this one runs)
    const float t = *a.tcall;
    for (uint32_t i = wave; i < nown; i += STG_WAVES) {  // overflowed lists: the chunk again (rare)
        const uint64_t off = before + s_off[i];
        if (s_cnt[i] > TV_CAPC && off < a.cap)
            tv_rescan(a.src, a.n, a.idx, a.val, c0 + i, off, (uint32_t)std::min<uint64_t>(s_cnt[i], a.cap - off), t);
    }
    if (!last) return;
    all = blk_sum64<STG_WAVES>(all, sh64);
    gm = wave_max(gm);
    if (lane == 0) sh[wave] = gm;
    __syncthreads();
    if (tid == 0) {
        uint32_t gb = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) gb = max(gb, sh[w]);
        const float gmax = a.n ? u2f(gb) : -1.f;
        float nt = t;
        if ((uint64_t)a.k > all) nt = (float)((double)t * 0.99);
        else if ((uint64_t)a.k < all) nt = (float)fma(0.01 * (double)all / (double)a.k, (double)gmax, (double)t);
        a.state->t = nt;
        a.state->init = 1;
        *a.count_out = ld_sc1(a.fail) ? POISON_COUNT : (uint32_t)std::min<uint64_t>(all, a.cap);
    }
}

}  // namespace

uint32_t tv_chunks(size_t n) { return (uint32_t)((n + TV_CH - 1) / TV_CH); }
uint32_t tv_list_words(size_t n) { return tv_chunks(n) * TV_CAPC * 2u; }

hipError_t launch_tv(const TvLaunch &a, const DevWS &ws, hipStream_t s) {
    if (a.first) {
        const uint32_t rank = (uint32_t)std::min<uint64_t>(a.k, a.n - 1);
        hipError_t e = launch_radix_select(a.src, a.n, 0xffffffffu, 0, rank, ws, a.num_cu, s);
        if (e != hipSuccess) return e;
        tv_init_state<<<1, 1, 0, s>>>(a.state, ws.rsel);
    }
    // tv_pass by default: 52 us at C3 against 65-70 us for the chunk launches
    // (STG_TV_PASS=0 selects them)
    static const bool old_pass = !(getenv("STG_TV_PASS") && atoi(getenv("STG_TV_PASS")) == 0);
    if (old_pass) return launch_tv_pass(a, ws, s);
    if (a.n >= (1ull << 32)) return hipErrorInvalidValue;  // positions are 32-bit
    TvcArgs f;
    f.src = a.src;
    f.n = a.n;
    f.nc = tv_chunks(a.n);
    f.k = a.k;
    f.cap = a.cap;
    f.idx = a.idx;
    f.val = a.val;
    f.count_out = a.count_out;
    f.state = a.state;
    f.lst = reinterpret_cast<uint2 *>(ws.sums);
    f.cnt = ws.tile_cnt;
    f.ng = (f.nc + TV_CPW - 1) / TV_CPW;
    if (f.ng > TV_MAXNG) return hipErrorInvalidValue;
    uint32_t *const gs = ws.tvg;  // [2 parities][sum, max][TV_MAXNG]
    const uint32_t par = a.par & 1u;
    f.gsum = gs + (2u * par) * TV_MAXNG;
    f.gmax = gs + (2u * par + 1u) * TV_MAXNG;
    f.zsum = gs + (2u * (par ^ 1u)) * TV_MAXNG;
    f.zmax = gs + (2u * (par ^ 1u) + 1u) * TV_MAXNG;
    f.zng = a.tv_ng[par ^ 1u];
    f.tcall = reinterpret_cast<float *>(gs + 4u * TV_MAXNG);  // the groups the other parity's last call used
    a.tv_ng[par] = f.ng;
    f.fail = ws.fail;
    const bool vec = (reinterpret_cast<uintptr_t>(a.src) & 15u) == 0;
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    // eight workgroups per CU, static contiguous chunk ranges (STG_TV_GPC: per CU)
    static const uint32_t gpc =
        getenv("STG_TV_GPC") ? (uint32_t)std::max(1, atoi(getenv("STG_TV_GPC"))) : (uint32_t)STG_TV_WPE;
    const uint32_t G = std::min<uint32_t>((f.nc + STG_WAVES - 1) / STG_WAVES, gpc * (uint32_t)std::max(a.num_cu, 1));
    if (vec) tv_chunk<true><<<G, STG_WG, 0, s>>>(f);
    else tv_chunk<false><<<G, STG_WG, 0, s>>>(f);
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    tv_fold<<<f.ng, STG_WG, 0, s>>>(f);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}

}  // namespace stg
