// tv16lf2.h -- the finish of a one-bucket thresholdv16 call inside its scan
// launch (tv16lone.hip), so that the common calls need no second launch's work.
// Included by tv16lone.hip in its anonymous namespace.
//
// Reference: ThresholdvCompressor16::impl_simd_v2 after the streaming
// (thresholdv16.cpp:138-259: emission order, stage 2's partial line, stage 3's
// ragged tail, AIMD) and the regime-B heap fill (:261-293).  The results are
// those of tv16lfin.h (the fill launch's finish of the same lists), which
// stays behind as the fallback.
//
// Arrival.  Each chunk's counts are stored last (sc1, after the lists are
// drained) and carry the call's tag.  The last F workgroups of the grid take
// the finisher roles once their own chunks are listed: they poll the chunks'
// counts until every one carries the tag (no counters: device-scope atomics on
// a shared word queue behind each other, ~0.3 us apiece here).  At most F
// workgroups of a call wait, and only for workgroups that run or have yet to
// start and never wait themselves.
//
// Roles (F of them, nwk workers first):
//   worker w   the qualifying lines of chunks [w pc, (w + 1) pc) at their
//              global ranks, from the scan's lists (no re-read of the bucket);
//              worker 0 also the ragged tail, the AIMD state and the count;
//   ranker r   in regime B, the kept window bins whose entries start in share
//              r of the kept entries: their order (sum desc, right-first
//              pre-order of the start position; tv16fill.hip (2), (3)), the
//              fast path's conditions, and their pops.  Every ranker loads all
//              kept entries (the tail's rank, the entry at rank Ph and the late
//              lines are global facts) and keeps its share in LDS.
// A role that cannot finish its part (a chunk whose lists overflowed, a window
// that does not hold the pops, a tie the fast path cannot order, a share past
// its LDS) does not count itself done, and the fill launch that follows
// finishes the call again from the same lists (its roles skip the call only
// when all F counted themselves done: tv16fill.hip).  Writing a result twice
// is harmless: both finishes write the same values.
#pragma once

#ifndef STG_LF2_STAMPS
#define STG_LF2_STAMPS 0  // diagnostics: phase stamps in debug words 0..15 (tools/lf2_probe.py)
#endif
#define LF2_STAMP(i)                                                                                 \
    do {                                                                                             \
        if (STG_LF2_STAMPS && threadIdx.x == 0) *gp(&A.dbg[(i)]) = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define LF2_STAMP_MAX(i)                                                                             \
    do {                                                                                             \
        if (STG_LF2_STAMPS && threadIdx.x == 0)                                                      \
            __hip_atomic_fetch_max(gp(&A.dbg[(i)]), (uint32_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
    } while (0)

constexpr uint32_t LF2_WG = 256;                    // the scan's workgroup
constexpr uint32_t LF2_NW = LF2_WG / 64;
constexpr uint32_t LF2_WK = 2048;                   // kept entries a ranker takes (8 per thread)
constexpr uint32_t LF2_KE = LF2_WK / LF2_WG;
constexpr uint32_t LF2_XB = LBCAP + 1;              // a special bin's entries (+ the tail)
constexpr uint32_t LF2_XC = 3 * LF2_XB;             // the special bins: the tail's, rank Ph's two candidates
constexpr uint32_t LF2_PER = LMAXC / LF2_WG;        // chunks per thread in the decision
constexpr uint32_t LF2_NONE = 0xffffffffu;
constexpr uint32_t LF2_POS_LIM = (1u << 20) - 1;    // rf_key's 20-bit paths
constexpr uint32_t LF2_TIES = 1u, LF2_VIOL = 2u;
constexpr uint32_t LF2_DBG_STALE = 31;            // debug word: workers the freshness check sent to the fill launch (tests read it)
constexpr uint32_t LF2_RC = 280;                    // a ranker's share of kept entries, at most
static_assert(LF2_KE * LF2_WG == LF2_WK && LF2_PER * LF2_WG == LMAXC, "per-thread counts");
static_assert(LNBIN == 4 * LF2_WG, "four bins per thread");

struct Lf2Args {
    const float *src;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    uint32_t nb, tl, dst_len, nc, fin, nwk, mode;
    int32_t idx_offset;
    const uint2 *ldesc;
    const uint32_t *lq;
    const uint2 *lw;
    const float4 *lv;
    const uint32_t *whist;
    const uint2 *went;
    KeyState *state;
    const CallParams *cp;
    float *resid;
    uint32_t *fail, *dbg, *done;
    uint32_t tag, skip;
    float t, inc;  // the key's state as this workgroup's scan read it (the state is updated only after every chunk)
};

struct Lf2Dec {
    uint32_t Qtot, Wtot, kb, r, lim, c0, ct, cnt, M, N;
    bool ok, regimeB, tail_cand, listw, lists_ok;  // ok: every chunk was listed in time
    float t, inc, tail_key;
};

struct Lf2Rk {
    uint64_t kg[LF2_RC];  // share entry -> (window offset << 25 | right-first key of its start position)
    uint32_t kc[LF2_RC];  // ... candidate index (start heap position)
    uint32_t kl[LF2_RC];  // ... line (the ragged tail: nb)
    uint16_t kb[LF2_RC];  // ... its bin
    uint16_t ord[LF2_RC]; // share rank -> share entry
    uint8_t tf[LF2_RC];   // ... tie flags
    uint64_t xg[LF2_XC];  // the special bins' entries (keys), LF2_XB per bin
    uint32_t late[64];    // start positions of R among the last Ph + 1
    uint32_t lc[64], lw[64];  // kept entries starting in the last Wk + 1 positions: start, window offset
};
struct Lf2Lds {
    Lf2Args a;
    uint32_t bin[LNBIN + 1];  // rankers: kept entries of the bins before each bin (+ all)
    uint16_t qp16[LMAXC];     // rankers: qualifying lines before each chunk (regime B: < 2^16)
    union {
        Lf2Rk r;
    } u;
    uint32_t sh[32];
    uint32_t v[16];
    float tail[16];
};

// 16-byte global stores through pointers taken from LDS (an address space the
// compiler cannot see: without the cast they become flat accesses, which count
// against lgkmcnt as well as vmcnt)
__device__ __forceinline__ void st_g16(void *p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    u4v v;
    v.x = a; v.y = b; v.z = c; v.w = d;
    *(__attribute__((address_space(1))) u4v *)p = v;
}

// 16 bytes at element `i` of `base` (uniform base), sc1
__device__ __forceinline__ float4 ld_sc1_f4(const float4 *base, uint32_t bytes, uint32_t i) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(base), 0, bytes, 0x00020000);
    const u4v t = __builtin_amdgcn_raw_buffer_load_b128(r, i * 16u, 0, 16 /* sc1 */);
    return make_float4(__uint_as_float(t.x), __uint_as_float(t.y), __uint_as_float(t.z), __uint_as_float(t.w));
}

// The decision every role takes: the chunks' counts (sc1, one round trip up to
// 2,048 chunks, repeated until every chunk carries the call's tag), the
// ragged tail (thread 0), then the regime as tv16.hip finish_chunk decides
// it.  Afterwards qp16[c] holds min(qualifying lines before chunk c, 65535):
// exact wherever it is below lim (lim = dst_len / 16 + 1 < 2^16 on this path,
// LMAXC chunks of LCHUNK lines, k <= n), which is all the roles use.
constexpr uint32_t kLf2PollSleep = 2;  // s_sleep between the finishers' descriptor polls (64 cycles a unit)
// Once every chunk's count pair carries the tag: ONE agent-scope acquire by
// one wave, its wait, then a workgroup barrier before any load of the lists
// (MI355X guide, "Valid forms", Consumer).  The lists are stored sc1 and
// loaded sc1, which the guide's table validates in place of the acquire only
// at one workgroup per CU; the scan runs eight per CU, so the acquire stays.
__device__ __forceinline__ void lf2_acquire() {
    if (threadIdx.x < 64) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}
template <bool WH>
__device__ __forceinline__ void lf2_decide(Lf2Lds &L, Lf2Dec &D, uint32_t (&h)[4]) {
    const Lf2Args &A = L.a;
    const uint32_t tid = threadIdx.x, nc = A.nc;
    constexpr uint32_t RH = LF2_PER / 2;  // loads per thread per round (chunk tid + 256 u)
    uint32_t sw = 0, bad = 0;
    D.ok = true;
    // (sc1 loads of the bucket: under the fused gather this launch wrote it)
    if (tid < A.tl) L.tail[tid] = u2f(ld_sc1(reinterpret_cast<const uint32_t *>(A.src) + (size_t)A.nb * 16 + tid));  // (in LDS: thread 0 sums them in order)
    const float t0 = A.t, i0 = A.inc;
    for (uint32_t h0 = 0; h0 * RH * LF2_WG < nc; ++h0) {
        uint64_t x[RH];
#pragma unroll
        for (uint32_t u = 0; u < RH; ++u) x[u] = 0;
        uint64_t st = 0;
        for (uint32_t sp = 0;; ++sp) {  // until every chunk of the round carries this call's tag
            uint32_t miss = 0;          // (a poll reloads only the chunks not yet seen listed)
#pragma unroll
            for (uint32_t u = 0; u < RH; ++u) {
                const uint32_t c = tid + (h0 * RH + u) * LF2_WG;
                if ((uint32_t)(x[u] >> 32) != A.tag)
                    x[u] = c < nc ? ld_sc1(reinterpret_cast<const uint64_t *>(A.ldesc) + c) : (uint64_t)A.tag << 32;
                miss |= (uint32_t)(x[u] >> 32) != A.tag ? 1u : 0u;
            }
            if (!__syncthreads_or((int)miss)) break;
            if (spin_expired(sp, st)) {
                if (tid == 0) { g_or(A.fail, FAIL_SPIN_TIMEOUT); st_sc1(A.count_out, POISON_COUNT); }
                D.ok = false;
                return;
            }
            __builtin_amdgcn_s_sleep(kLf2PollSleep);
        }
        if ((h0 + 1) * RH * LF2_WG >= nc) lf2_acquire();  // every chunk listed
        if (WH && (h0 + 1) * RH * LF2_WG >= nc) {  // the window histogram is final
#pragma unroll
            for (uint32_t u = 0; u < 4; ++u) h[u] = ld_sc1(&A.whist[whist_word(4 * tid + u)]);
        }
#pragma unroll
        for (uint32_t u = 0; u < RH; ++u) {
            const uint32_t c = tid + (h0 * RH + u) * LF2_WG;
            const uint32_t q = (uint32_t)x[u] & 0xffffu, w = ((uint32_t)x[u] >> 16) & 0xffffu;
            sw += w;
            bad |= (q > LQCAP || w > LWCAP) ? 1u : 0u;
            if (c < nc) L.qp16[c] = (uint16_t)q;  // (a chunk has <= LCHUNK lines)
        }
    }
    __syncthreads();
    // exclusive prefixes, LF2_PER consecutive chunks per thread
    uint32_t s = 0;
#pragma unroll
    for (uint32_t u = 0; u < LF2_PER; ++u) {
        const uint32_t c = tid * LF2_PER + u;
        s += c < nc ? L.qp16[c] : 0u;
    }
    D.t = t0;
    D.inc = i0;
    uint32_t pq = blk_excl_scan<LF2_NW>(s, L.sh, &D.Qtot);
    (void)blk_excl_scan<LF2_NW>(sw, L.sh, &D.Wtot);
#pragma unroll
    for (uint32_t u = 0; u < LF2_PER; ++u) {
        const uint32_t c = tid * LF2_PER + u;
        if (c >= nc) break;
        const uint32_t q = L.qp16[c];
        L.qp16[c] = (uint16_t)min(pq, 0xffffu);
        pq += q;
    }
    D.lists_ok = !__syncthreads_or((int)bad);
    const uint32_t Qtot = D.Qtot, dst_len = A.dst_len;
    D.kb = dst_len / 16;
    D.r = dst_len % 16;
    D.lim = D.kb + (D.r ? 1u : 0u);
    D.c0 = Qtot >= D.lim ? dst_len : 16u * Qtot;
    if (tid == 0) {  // stage 3: the ragged tail's signed, sequential sum (thresholdv16.cpp:212-236)
        uint32_t ct = 0, cand = 0;
        float key = 0.f;
        if (D.c0 < dst_len && A.tl) {
            float sm = 0.f;
            for (uint32_t i = 0; i < A.tl; ++i) sm += L.tail[i];
            if (sm * 16.0f >= D.t * (float)A.tl) ct = min(dst_len - D.c0, A.tl);
            else { cand = 1; key = sm * 16.0f / (float)A.tl; }
        }
        L.v[0] = ct;
        L.v[1] = cand;
        L.v[2] = f2u(key);
    }
    __syncthreads();
    D.ct = L.v[0];
    D.tail_cand = L.v[1] != 0;
    D.tail_key = u2f(L.v[2]);
    __syncthreads();
    D.cnt = D.c0 + D.ct;
    D.regimeB = D.cnt < dst_len;
    const uint32_t ncand = A.nb - Qtot;  // non-qualifying full lines
    D.M = D.regimeB ? min((dst_len - D.cnt + 15u) / 16u, ncand) : 0u;
    D.listw = D.regimeB && D.Wtot >= D.M && D.Wtot + 1 <= CAND_CAP;
    D.N = ncand + (D.tail_cand ? 1u : 0u);  // the reference's candidate vector length
}

// one quarter (four floats) of a qualifying line at its global rank g (lfin_store)
__device__ __forceinline__ void lf2_store(const Lf2Args &A, bool vec, uint32_t g, uint32_t kb, uint32_t r, uint32_t line,
                                          float4 x, uint32_t q) {
    const uint32_t len = g == kb ? r : 16u, off = 16 * g + 4 * q, pos = line * 16 + 4 * q;
    const uint32_t bi = pos + (uint32_t)A.idx_offset;
    if (vec && len == 16) {
        st_g16(A.idx + off, bi, bi + 1, bi + 2, bi + 3);
        st_g16(A.val + off, __float_as_uint(x.x), __float_as_uint(x.y), __float_as_uint(x.z), __float_as_uint(x.w));
    } else {
        const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc)
            if (4 * q + cc < len) { *gp(A.idx + off + cc) = bi + cc; *gp(A.val + off + cc) = xs[cc]; }
    }
}

__device__ __forceinline__ bool lf2_aligned(const Lf2Args &A) {
    return ((reinterpret_cast<uintptr_t>(A.src) | reinterpret_cast<uintptr_t>(A.idx) |
             reinterpret_cast<uintptr_t>(A.val)) & 15u) == 0;
}

// ---------------------------------------------------------------------------
// worker `wk`: true when its share is written
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool lf2_worker(Lf2Lds &L, uint32_t wk) {
    const Lf2Args &A = L.a;
    const uint32_t tid = threadIdx.x, nc = A.nc, nwk = A.nwk;
    Lf2Dec D;
    uint32_t h[4];
    lf2_decide<false>(L, D, h);
    if (wk == 0) LF2_STAMP(3);
    if (!D.ok || !D.lists_ok || D.lim > 0xffffu) return false;  // (lists overflowed: the fill launch re-reads them)
    if (A.skip == 4) return false;
    // static map: the workers' threads, TPC per chunk (no prefix over the
    // workers' chunks to build); thread sub of chunk c takes the quarter lines
    // sub, sub + TPC, ... of the chunk's lines below lim
    const uint32_t gt = wk * LF2_WG + tid, tpc = max(1u, nwk * LF2_WG / nc), c = gt / tpc, sub = gt % tpc;
    const bool vec = lf2_aligned(A);
    const uint32_t lv_bytes = nc * LQCAP * 4u * 16u, tag16 = A.tag & 0xffffu;
    uint32_t stale = 0;  // a listed line without this call's tag (tv16lone.hip finalize)
    if (wk == 0) LF2_STAMP(20);
    for (uint32_t cc = c; cc < nc; cc += nwk * LF2_WG / tpc) {  // (one pass unless nc > nwk LF2_WG)
        const uint32_t g0 = L.qp16[cc];
        if (g0 >= D.lim) continue;
        const uint32_t g1 = cc + 1 < nc ? L.qp16[cc + 1] : min(D.Qtot, 0xffffu);
        const uint32_t ne = 4u * min(g1 - g0, D.lim - g0);  // quarter lines to emit
        constexpr uint32_t K = 4;
        for (uint32_t t0 = sub; t0 < ne; t0 += K * tpc) {
            float4 x[K];
            uint32_t ln[K];
#pragma unroll
            for (uint32_t j = 0; j < K; ++j) {
                const uint32_t t = t0 + j * tpc, sl = t >> 2;
                if (t < ne) {
                    ln[j] = ld_sc1(&A.lq[(size_t)cc * LQCAP + sl]);
                    x[j] = ld_sc1_f4(A.lv, lv_bytes, (cc * LQCAP + sl) * 4u + (t & 3u));
                }
            }
            if (STG_LF2_STAMPS && wk == 0 && cc == c && t0 == sub) { vm_drain(); LF2_STAMP(21); }
#pragma unroll
            for (uint32_t j = 0; j < K; ++j) {
                const uint32_t t = t0 + j * tpc;
                if (t < ne) {
                    stale |= (ln[j] >> 16) != tag16 ? 1u : 0u;
                    lf2_store(A, vec, g0 + (t >> 2), D.kb, D.r, cc * LCHUNK + (ln[j] & 0xffffu), x[j], t & 3u);
                }
            }
        }
    }
    // Consistency: every list entry this worker emitted must carry the call's
    // tag.  One that does not means a list read before its chunk's stores were
    // visible (or a count pair not from this call): the worker does not count
    // itself done, and the fill launch, after the kernel boundary, emits the
    // call again from the same lists.
    if (__syncthreads_or((int)stale)) {
        if (tid == 0) g_add(&A.dbg[LF2_DBG_STALE], 1u);
        return false;
    }
    // worker 0: tail, AIMD state, count (tv16.hip finish_chunk, lfin_worker)
    if (wk == 0 && tid == 0) {
        const size_t p0 = (size_t)A.nb * 16;
        for (uint32_t i = 0; i < D.ct; ++i) {
            *gp(A.idx + D.c0 + i) = (uint32_t)(p0 + i) + (uint32_t)A.idx_offset;
            *gp(A.val + D.c0 + i) = u2f(ld_sc1(reinterpret_cast<const uint32_t *>(A.src) + p0 + i));
        }
        if (A.resid)  // fused error feedback: the ragged tail is not streamed
            for (uint32_t i = 0; i < A.tl; ++i)
                *gp(A.resid + p0 + i) = u2f(ld_sc1(reinterpret_cast<const uint32_t *>(A.src) + p0 + i));
        auto st = gp(A.state);
        st->t = D.regimeB ? (float)((double)D.t * 0.99) : D.t + D.inc;  // thresholdv16.cpp:243-259
        st->inc = D.inc;
        st->init = 1;
        st_sc1(A.count_out, (uint32_t)min((uint64_t)A.dst_len, (uint64_t)A.nb * 16 + A.tl));
        if (ld_sc1(A.fail)) st_sc1(A.count_out, POISON_COUNT);
    }
    if (wk == 0) LF2_STAMP(4);
    return true;
}

// ---------------------------------------------------------------------------
// ranker `rk` of NR: true when its share of the regime-B fill is written in
// the reference's pop order (or there is no fill)
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool lf2_ranker(Lf2Lds &L, uint32_t rk) {
    const Lf2Args &A = L.a;
    const uint32_t tid = threadIdx.x, NR = A.fin - A.nwk;
    Lf2Dec D;
    uint32_t h[4];  // the scan's window entries per bin (loaded once every chunk is listed)
    lf2_decide<true>(L, D, h);
    if (!D.ok) return false;
    if (rk == 0) LF2_STAMP(5);
    auto fail_at = [&](uint32_t why) {
        if (STG_LF2_STAMPS && rk == 0 && tid == 0) { A.dbg[7] = why; A.dbg[11] = (uint32_t)__builtin_amdgcn_s_memrealtime(); }
        return false;
    };
    if (!D.regimeB || (!D.M && !D.tail_cand)) return true;  // nothing to fill
    const uint32_t tb = f2u(D.t), wlo = tb > TV16_WIN ? tb - TV16_WIN : 0u;
    const bool tail_in = D.tail_cand && D.tail_key >= u2f(wlo);
    const uint32_t W = D.Wtot + (tail_in ? 1u : 0u);
    // (the conditions of lfin_ranker; a -0.0 tail ties +0.0 sums in the
    // reference's float compare, not in this key order; prefixes fit u16)
    if (!D.listw || !D.lists_ok || D.N > LF2_POS_LIM || W == 0 || A.mode || D.Qtot > 0xffffu ||
        (tail_in && (f2u(D.tail_key) & 0x80000000u)) || (tail_in && !(D.tail_key < D.t)))
        return fail_at(1);
    const uint32_t tw = tail_in ? tb - 1u - f2u(D.tail_key) : 0u, tbin = tail_in ? tw >> 8 : LF2_NONE;
    const uint32_t need = D.M + 2, rem = A.dst_len - D.cnt;
    // ---- bin starts; the first bins holding need entries are kept ----
    {
        uint32_t c[4], s = 0;
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            c[u] = h[u] + (4 * tid + u == tbin ? 1u : 0u);
            s += c[u];
        }
        uint32_t tot;
        uint32_t run = blk_excl_scan<LF2_NW>(s, L.sh, &tot);
#pragma unroll
        for (uint32_t u = 0; u < 4; ++u) {
            const uint32_t b = 4 * tid + u;
            L.bin[b] = run;
            if (run < need && run + c[u] >= need) { L.v[3] = b + 1; L.v[4] = run + c[u]; }
            run += c[u];
        }
        if (tid == 0) {
            L.bin[LNBIN] = tot;
            if (tot < need) { L.v[3] = LNBIN; L.v[4] = tot; }
            L.v[8] = 0;      // late lines
            L.v[7] = 0;      // late candidates
        }
        __syncthreads();
    }
    if (rk == 0) LF2_STAMP(2);
    if (A.skip == 1) return false;
    const uint32_t cut = L.v[3], Wk = L.v[4];
    bool over = false;
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) over |= (4 * tid + u < cut && h[u] > LBCAP);
    if (__syncthreads_or((int)over) || Wk > LF2_WK || Wk == 0 || 16u * Wk < rem) return fail_at(2);
    // ---- one parallel pass (every thread its four bins and its chunks, no
    //      dependent searches): this ranker's bins [b_lo, b_hi) (the first bins
    //      starting at or past ceil(rk Wk / NR) and ceil((rk + 1) Wk / NR)), the
    //      bins holding ranks ra and rb (rank Ph's candidates), and the first
    //      chunk that may hold a candidate position >= late_min ----
    const uint32_t P0 = (rem + 15u) / 16u;
    const uint32_t ra = min(P0 + 1u, Wk - 1u), rb = min(P0 + 2u, Wk - 1u);
    const uint32_t x_lo = (uint32_t)(((uint64_t)rk * Wk + NR - 1) / NR), x_hi = (uint32_t)(((uint64_t)(rk + 1) * Wk + NR - 1) / NR);
    const uint32_t late_min = D.N > Wk + 1 ? D.N - (Wk + 1) : 0u;
    if (tid == 0) { L.v[5] = x_lo ? cut : 0u; L.v[6] = x_hi ? cut : 0u; }
    __syncthreads();
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t b = 4 * tid + u;
        if (b >= cut) continue;
        const uint32_t sb = L.bin[b], eb = L.bin[b + 1];
        if (x_lo && sb < x_lo && eb >= x_lo) L.v[5] = b + 1;  // (the first bin starting >= x_lo is b + 1)
        if (x_hi && sb < x_hi && eb >= x_hi) L.v[6] = b + 1;
        if (sb <= ra && ra < eb) L.v[14] = b;
        if (sb <= rb && rb < eb) L.v[15] = b;
    }
    if (tid < 64) {  // the predicate (c + 1) LCHUNK - 1 - qp[c] >= late_min rises once, within the last 64 chunks
        const uint32_t c = A.nc - 1u - tid;
        const bool pc = tid < A.nc && (c + 1u) * LCHUNK - 1u - L.qp16[c] >= late_min;
        const uint64_t bl = __ballot(pc);  // lanes 0 .. j - 1 hold the chunks at or past the rise
        const uint32_t j = (uint32_t)__popcll(bl);
        if (tid == 0 && bl == (j == 64 ? ~0ull : ((1ull << j) - 1ull))) L.v[9] = A.nc - j;
        else if (tid == 0) L.v[9] = 0;  // (not one rise in the last 64 chunks: fails below)
    }
    __syncthreads();
    const uint32_t b_lo = L.v[5], b_hi = L.v[6], sb1 = L.v[14], sb2 = L.v[15], cf = L.v[9];
    const uint32_t E0 = L.bin[b_lo], E1 = L.bin[b_hi], ne = E1 - E0;
    if (STG_LF2_STAMPS && rk == 0 && tid == 0) { A.dbg[12] = Wk; A.dbg[13] = ne; }
    if (ne > LF2_RC) return fail_at(3);
    const uint32_t sb0 = tbin < cut ? tbin : LF2_NONE;
    auto is_tail = [&](uint32_t e, uint32_t b) { return b == tbin && e + 1 == L.bin[b + 1]; };
    // the share's entries' bins (from its bins, a few entries each)
#pragma unroll
    for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t b = 4 * tid + u;
        if (b >= b_lo && b < b_hi) {
            const uint32_t e0 = L.bin[b], e1 = L.bin[b + 1];
            for (uint32_t e = e0; e < e1; ++e) L.u.r.kb[e - E0] = (uint16_t)b;
        }
    }
    __syncthreads();
    // ---- loaded together: the share's entries (<= 2 per thread), the special
    //      bins' entries (<= 1 per thread) and the window lists of the last
    //      chunks (the lines that may start in the last Wk + 1 positions: the
    //      late lines of R are among them) ----
    if ((A.nc - cf) * LWCAP > LF2_WG) return fail_at(7);
    {
        const uint64_t *const went = reinterpret_cast<const uint64_t *>(A.went);
        // own entries
        uint32_t bj[2];
        uint64_t y[2];
#pragma unroll
        for (uint32_t j = 0; j < 2; ++j) bj[j] = tid + j * LF2_WG < ne ? L.u.r.kb[tid + j * LF2_WG] : b_lo;
#pragma unroll
        for (uint32_t j = 0; j < 2; ++j) {
            const uint32_t i = tid + j * LF2_WG, e = E0 + i;
            y[j] = 0;
            if (i < ne && !is_tail(e, bj[j])) y[j] = ld_sc1(went + bj[j] * LBCAP + (e - L.bin[bj[j]]));
        }
        // special bins: thread t -> bin k = t / LF2_XB, entry t % LF2_XB
        const uint32_t k = tid / LF2_XB, xi = tid % LF2_XB;
        const uint32_t sbk = k == 0 ? sb0 : k == 1 ? sb1 : k == 2 ? sb2 : LF2_NONE;
        const bool xin = sbk != LF2_NONE && xi < L.bin[sbk + 1] - L.bin[sbk];
        uint64_t yx = 0;
        if (xin && !is_tail(L.bin[sbk] + xi, sbk)) yx = ld_sc1(went + sbk * LBCAP + xi);
        // the last chunks' window lists and their counts
        const uint32_t lc_c = cf + tid / LWCAP, lc_s = tid % LWCAP;
        uint64_t yl = 0, dl = 0;
        if (lc_c < A.nc) {
            dl = ld_sc1(reinterpret_cast<const uint64_t *>(A.ldesc) + lc_c);
            yl = ld_sc1(reinterpret_cast<const uint64_t *>(A.lw) + (size_t)lc_c * LWCAP + lc_s);
        }
        if (A.skip == 2) { vm_drain(); return false; }
        if (STG_LF2_STAMPS && rk == 0) { vm_drain(); LF2_STAMP(11); }
        auto decode = [&](uint64_t v, uint32_t &w, uint32_t &cx, uint32_t &line) {  // a binned window entry
            const uint32_t sx = (uint32_t)v, yy = (uint32_t)(v >> 32), c = yy >> 19;
            line = c * LCHUNK + ((yy >> 10) & 511u);
            w = tb - 1u - sx;
            cx = line - ((uint32_t)L.qp16[c] + (yy & 1023u));
        };
#pragma unroll
        for (uint32_t j = 0; j < 2; ++j) {
            const uint32_t i = tid + j * LF2_WG, e = E0 + i;
            if (i >= ne) continue;
            uint32_t w, cx, line;
            if (is_tail(e, bj[j])) {  // the candidate vector's last entry (thresholdv16.cpp:229-234)
                w = tw;
                cx = D.N - 1;
                line = A.nb;
            } else {
                decode(y[j], w, cx, line);
            }
            L.u.r.kg[i] = (uint64_t)w << 25 | rf_key(cx);
            L.u.r.kc[i] = cx;
            L.u.r.kl[i] = line;
            L.u.r.kb[i] = (uint16_t)bj[j];
        }
        if (xin) {
            uint32_t w, cx, line;
            if (is_tail(L.bin[sbk] + xi, sbk)) { w = tw; cx = D.N - 1; }
            else decode(yx, w, cx, line);
            L.u.r.xg[k * LF2_XB + xi] = (uint64_t)w << 25 | rf_key(cx);
        }
        // late candidates: window lines of the last chunks starting at >= late_min, and the tail
        if (lc_c < A.nc && lc_s < (((uint32_t)dl >> 16) & 0xffffu) && lc_s < LWCAP) {
            const uint32_t sx = (uint32_t)yl, yy = (uint32_t)(yl >> 32);
            const uint32_t line = lc_c * LCHUNK + (yy & 0xffffu);
            const uint32_t cx = line - ((uint32_t)L.qp16[lc_c] + (yy >> 16)), w = tb - 1u - sx;
            if (cx >= late_min && cx) {
                const uint32_t i = atomicAdd(&L.v[7], 1u);
                if (i < 64) { L.u.r.lc[i] = cx; L.u.r.lw[i] = w; }
            }
        }
        if (tid == 0 && tail_in && D.N - 1 >= late_min && D.N > 1) {
            const uint32_t i = atomicAdd(&L.v[7], 1u);
            if (i < 64) { L.u.r.lc[i] = D.N - 1; L.u.r.lw[i] = tw; }
        }
    }
    __syncthreads();
    if (rk == 0) LF2_STAMP(10);
    if (A.skip == 3) return false;
    // ---- at once: wave 0 takes the global facts from the special bins (the
    //      tail's rank tr, the pops P, Ph and the window offset wh of the entry
    //      at rank Ph: R = offsets <= wh); every thread ranks its share entries
    //      (bins lie whole in the share, so an entry's rank is its bin's start
    //      plus the bin's smaller keys; ties, equal offsets, noted) ----
    if (tid < 64) {
        const uint32_t lane = tid;
        // each lane holds one entry of a special bin; its rank in the bin by
        // comparing with every lane's entry (read lanes: no LDS round trips)
        auto inbin_rank = [&](uint32_t k, uint32_t n, uint64_t &g) {
            g = lane < n ? L.u.r.xg[k * LF2_XB + lane] : ~0ull;
            const uint32_t glo = (uint32_t)g, ghi = (uint32_t)(g >> 32);
            uint32_t r = 0;
            for (uint32_t x = 0; x < n; ++x) {
                const uint32_t xl = (uint32_t)__builtin_amdgcn_readlane((int)glo, (int)x);
                const uint32_t xh = (uint32_t)__builtin_amdgcn_readlane((int)ghi, (int)x);
                r += (xh < ghi || (xh == ghi && xl < glo)) ? 1u : 0u;
            }
            return r;
        };
        uint32_t tr = LF2_NONE;  // the tail is its bin's last entry
        if (sb0 != LF2_NONE) {
            const uint32_t n = L.bin[sb0 + 1] - L.bin[sb0];
            uint64_t g;
            const uint32_t r = inbin_rank(0, n, g);
            tr = L.bin[sb0] + (uint32_t)__builtin_amdgcn_readlane((int)r, (int)(n - 1));
        }
        uint32_t P = P0;
        if (tr < P) P = (rem + (16u - A.tl) + 15u) / 16u;
        P = min(P, Wk);
        const uint32_t Ph = min(P + 1, Wk - 1);
        const uint32_t k = Ph == ra ? 1u : 2u, b = k == 1 ? sb1 : sb2, n = L.bin[b + 1] - L.bin[b];
        const uint32_t want = Ph - L.bin[b];
        // the bin's entries are distinct keys: exactly one has `want` smaller
        uint64_t g;
        const uint32_t r = inbin_rank(k, n, g);
        uint32_t hit = (lane < n && r == want) ? (uint32_t)(g >> 25) + 1u : 0u;
        hit = wave_max(hit);
        if (lane == 0) {
            L.v[9] = tr;
            L.v[10] = P;
            L.v[11] = Ph;
            L.v[12] = hit ? hit - 1u : 0u;  // wh
            L.v[13] = hit ? 1u : 0u;
        }
    }
    for (uint32_t i = tid; i < ne; i += LF2_WG) {
        const uint32_t b = L.u.r.kb[i], lo = L.bin[b] - E0, hi = L.bin[b + 1] - E0;
        const uint64_t ge = L.u.r.kg[i];
        const uint32_t we = (uint32_t)(ge >> 25);
        uint32_t r = lo;
        bool tie = false;
        for (uint32_t x = lo; x < hi; ++x) {
            const uint64_t gx = L.u.r.kg[x];
            r += gx < ge;
            tie |= (uint32_t)(gx >> 25) == we && gx != ge;
        }
        uint32_t f = 0;
        if (tie) {  // rare: is a tied line's start below this one's?
            f = LF2_TIES;
            const uint32_t qe = L.u.r.kc[i] + 1;
            for (uint32_t x = lo; x < hi; ++x)
                if (x != i && (uint32_t)(L.u.r.kg[x] >> 25) == we && is_desc(L.u.r.kc[x] + 1, qe)) f |= LF2_VIOL;
        }
        L.u.r.tf[i] = (uint8_t)f;
        L.u.r.ord[r] = (uint16_t)i;
    }
    __syncthreads();
    if (rk == 0) LF2_STAMP(14);
    const uint32_t tr = L.v[9], P = L.v[10], Ph = L.v[11], wh = L.v[12];
    if (!L.v[13] || (tr != LF2_NONE && 16u * Wk - (16u - A.tl) < rem)) return fail_at(4);
    const uint32_t late = D.N > Ph + 1 ? D.N - (Ph + 1) : 0u;  // start positions >= late: the last Ph + 1
    if (L.v[7] > 64) return fail_at(5);  // (every ranker sees the same count)
    // ---- the share's pops (ranks [E0, min(E1, P)), four lanes per line):
    //      their loads go out now, the stores wait for the checks ----
    const bool vec = lf2_aligned(A) && (D.cnt & 3u) == 0;
    const uint32_t src_bytes = A.nb * 64u;  // the full lines (< 2^32 bytes: LMAXC chunks of LCHUNK lines)
    const uint32_t s1 = min(E1, P), q = tid & 3u;
    constexpr uint32_t LPR = LF2_WG / 4, NRD = 2;
    float4 v[NRD];
    uint32_t pos[NRD], off[NRD], len[NRD];
    auto load_round = [&](uint32_t j0) {
#pragma unroll
        for (uint32_t u = 0; u < NRD; ++u) {
            const uint32_t i = j0 + u * LPR + (tid >> 2);
            len[u] = 0;
            v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (i < s1) {
                off[u] = 16u * i - (tr < i ? 16u - A.tl : 0u);
                if (off[u] < rem) {
                    len[u] = min(i == tr ? A.tl : 16u, rem - off[u]);
                    pos[u] = L.u.r.kl[L.u.r.ord[i - E0]] * 16u;
                    if (vec && len[u] == 16 && (off[u] & 3u) == 0) v[u] = ld_sc1_f4(reinterpret_cast<const float4 *>(A.src), src_bytes, pos[u] / 4 + q);
                }
            }
        }
    };
    auto store_round = [&]() {
#pragma unroll
        for (uint32_t u = 0; u < NRD; ++u) {
            if (!len[u]) continue;
            const uint32_t o = D.cnt + off[u] + 4 * q, bi = pos[u] + 4 * q + (uint32_t)A.idx_offset;
            if (vec && len[u] == 16 && (off[u] & 3u) == 0) {
                st_g16(A.idx + o, bi, bi + 1, bi + 2, bi + 3);
                st_g16(A.val + o, __float_as_uint(v[u].x), __float_as_uint(v[u].y), __float_as_uint(v[u].z),
                       __float_as_uint(v[u].w));
            } else {
                for (uint32_t cc = 0; cc < 4; ++cc)
                    if (4 * q + cc < len[u]) {
                        *gp(A.idx + o + cc) = bi + cc;
                        *gp(A.val + o + cc) = u2f(ld_sc1(reinterpret_cast<const uint32_t *>(A.src) + (size_t)pos[u] + 4 * q + cc));
                    }
            }
        }
    };
    load_round(E0);
    // ---- the late lines of R, from the late candidates ----
    if (tid < L.v[7] && L.u.r.lw[tid] <= wh && L.u.r.lc[tid] >= late) {
        const uint32_t i = atomicAdd(&L.v[8], 1u);
        L.u.r.late[i] = L.u.r.lc[tid];
    }
    __syncthreads();
    // ---- the fast path's conditions (tv16fill.hip (3)) for the share's R ----
    uint32_t fl = 0;
    const uint32_t nl = L.v[8];
    if (nl > 64) fl |= LF2_VIOL;
    for (uint32_t i = tid; i < ne; i += LF2_WG) {
        if ((uint32_t)(L.u.r.kg[i] >> 25) > wh) continue;
        fl |= L.u.r.tf[i];
        const uint32_t cf = L.u.r.kc[i];
        for (uint32_t x = 0; x < min(nl, 64u); ++x) {
            const uint32_t ce = L.u.r.late[x];
            if (cf == (ce - 1) / 2 || cf == ((ce - 1) ^ 1u) + 1) fl |= LF2_VIOL;
        }
    }
    const bool viol = __syncthreads_or((int)(fl & LF2_VIOL));
    const bool ties = __syncthreads_or((int)(fl & LF2_TIES));
    if (viol) return fail_at(6);
    if (rk == 0) LF2_STAMP(6);
    store_round();
    for (uint32_t j0 = E0 + NRD * LPR; j0 < s1; j0 += NRD * LPR) {
        load_round(j0);
        store_round();
    }
    if (rk == 0 && tid == 0) g_add(&A.dbg[ties ? 45 : 44], 1u);  // calls ranked in the scan launch
    if (rk == 0) LF2_STAMP(8);
    return true;
}

// After the chunk loop, in the last F workgroups of the grid: role `role`.
__device__ __forceinline__ void lf2_finish(Lf2Lds &L, const LScanArgs &A, uint32_t role, float t, float inc) {
    const uint32_t tid = threadIdx.x;
    __syncthreads();  // every wave is out of the chunk loop: the LDS goes to the finish
    if (tid == 0) {
        // the arguments the roles take (by reference from LDS: a reference to
        // the kernel's argument block would be copied to scratch)
        Lf2Args &a = L.a;
        a.src = A.src;
        a.idx = A.out_idx;
        a.val = A.out_val;
        a.count_out = A.count_out;
        a.nb = A.nb;
        a.tl = A.tl;
        a.dst_len = A.dst_len;
        a.nc = A.nc;
        a.fin = A.fin;
        a.nwk = A.nwk;
        a.mode = A.mode;
        a.idx_offset = A.idx_offset;
        a.ldesc = A.ldesc;
        a.lq = A.lq;
        a.lw = A.lw;
        a.lv = A.lv;
        a.whist = A.whist;
        a.went = A.went;
        a.state = A.state;
        a.cp = A.cp;
        a.resid = A.resid;
        a.fail = A.fail;
        a.dbg = A.dbg;
        a.done = A.done;
        a.tag = A.tag;
        a.skip = A.skip;
        a.t = t;
        a.inc = inc;
    }
    __syncthreads();
    if (role == 0) LF2_STAMP_MAX(1);
    const bool ok = role < L.a.nwk ? lf2_worker(L, role) : lf2_ranker(L, role - L.a.nwk);
    // the role's part is written (the fill launch reads the flag after this
    // launch has ended: every store is visible then)
    __syncthreads();
    if (ok && tid == 0) st_sc1(&A.done[role], A.tag);
    LF2_STAMP_MAX(9);  // the last role's end
}
