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
// GPU structure: one launch, HBM-bound (tv_pass).  1024-thread workgroups
// (kTvWpc per CU) take contiguous ranges of the bucket in ticket order; 16 waves
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

constexpr uint32_t kTvTwg = 1024;
constexpr uint32_t TWG = kTvTwg;  // threads per workgroup (16 waves)
constexpr uint32_t TNW = TWG / 64;
constexpr uint32_t kTvWpc = 1;  // workgroups per CU (1 with 6 loads in flight per lane: 52.3 us at C3; 2 with 4: 55.6)
constexpr uint32_t kTvScanD = 6;
constexpr uint32_t SCAN_D = kTvScanD;  // float4 loads in flight per lane
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
    // kTvWpc workgroups per CU, each with >= 64 KiB of the bucket
    const uint64_t n4 = a.n / 4;
    const uint32_t G = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>(std::min<uint64_t>((uint64_t)kTvWpc * a.num_cu, TV_MAXG), (n4 + 4095) / 4096));
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


}  // namespace

hipError_t launch_tv(const TvLaunch &a, const DevWS &ws, hipStream_t s) {
    if (a.first) {
        const uint32_t rank = (uint32_t)std::min<uint64_t>(a.k, a.n - 1);
        hipError_t e = launch_radix_select(a.src, a.n, 0xffffffffu, 0, rank, ws, a.num_cu, s);
        if (e != hipSuccess) return e;
        tv_init_state<<<1, 1, 0, s>>>(a.state, ws.rsel);
    }
    return launch_tv_pass(a, ws, s);
}

}  // namespace stg
