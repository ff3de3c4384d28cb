// tv16lfin.h -- the finish of a one-bucket thresholdv16 scan (tv16lone.hip),
// inside the fill launch (tv16fill.hip, lfin mode).  Included by tv16fill.hip
// in its anonymous namespace, after FillLds and the fill's helpers.
//
// Reference: ThresholdvCompressor16::impl_simd_v2 after the streaming
// (thresholdv16.cpp:138-259: emission order, stage 2's partial line, stage 3's
// ragged tail, AIMD) and the regime-B heap fill (:261-293).
//
// The scan left per chunk of LCHUNK lines its counts (ldesc), its qualifying
// lines in order with their data (lq, lv) and its window lines in order (lw:
// {sum bits, line within the chunk | qualifying lines before it << 16}).
// Three roles share the launch, none waits on another:
//   workers  (tickets [0, workers))  take the chunks' prefix counts, decide
//            the regime exactly as the batched scan's last chunk does
//            (tv16.hip finish_chunk), write a balanced share of the
//            qualifying lines at their global ranks and of the window list in
//            scan order (the exact orderer's input); worker 0 writes the
//            ragged tail, the AIMD state, the count and the decision;
//   rankers  (the next `rankers` tickets)  decide the same way; in regime B
//            each reads the scan's window histogram (ws.h LNBIN bins of 256
//            ulps below t), keeps the first bins (the pops, the first line
//            past them and its ties), loads only those bins' entries (the scan
//            stored them by bin), ranks every kept line by (sum desc,
//            right-first pre-order of the start position) -- the pop order
//            whenever the fill's fast paths hold (see tv16fill.hip (2), (3))
//            -- checks those conditions, and emits its share of the pops;
//   every workgroup then adds to one counter; the last one (every write of
//            the others is in) runs the exact orderer of tv16fill.hip over the
//            workers' window list when the rankers could not prove their
//            order (a violation among ties, a window the scan's lists could
//            not hold, or the window missed the top), overwriting the fill.
#pragma once

// LDS of the lfin roles (a view of the launch's dynamic LDS, like FillLds).
struct LfinArgs {
    Tv16FillBucket d;
    uint32_t nc, workers, rankers, epoch, mode;
    const uint2 *ldesc;
    const uint32_t *lq;
    const uint2 *lw;
    const float4 *lv;
    uint32_t *whist;  // the scan's binned window: counts per bin, entries LBCAP per bin
    const uint2 *went;
    KeyState *state;
    const CallParams *cp;
    float *resid;
    uint32_t *fail;
    Decision *dec;
    CallCtl *cc;
    uint32_t *dbg;  // diagnostics: lfin counters at words 48..55, ranker 0's phase stamps at 32..47
};
constexpr uint32_t LF_QMAP = 8192;  // worker: ranks mapped to their chunk per pass
struct LfinLds {
    uint32_t qp[LMAXC + 1];  // per chunk: exclusive prefix of qualifying lines (+ total)
    uint32_t wp[LMAXC + 1];  // ... of window lines
    union {
        struct {                       // ranker: the kept window entries, grouped by bin
            uint64_t kg[EMAX];         // sort key: window offset (bits(t) - 1 - bits(sum)) << 25 | right-first key
            uint32_t kc[EMAX];         // ... candidate index (start heap position)
            uint32_t kl[EMAX];         // ... line (the ragged tail: nb)
            uint16_t emap[EMAX];       // ... its bin
            uint16_t ord[EMAX];        // rank -> kept entry
            uint8_t tf[EMAX];          // ... LF_TIES / LF_VIOL if it turns out to be in R
        } r;
        struct {                       // worker: rank -> chunk
            uint16_t qmap[LF_QMAP];
        } w;
    } u;
    uint32_t bin[NBIN + 1];    // ranker: kept entries of the bins before each bin (+ all)
    uint32_t sh[32];
    uint32_t late[64];         // lines of R starting in the last Ph + 1 positions
    uint32_t cut, wk, tail_rank, nlate;
    LfinArgs args;
};

__device__ __forceinline__ uint32_t chunk_of(const uint32_t *p, uint32_t nc, uint32_t g) {
    uint32_t lo = 0, hi = nc;  // the last c < nc with p[c] <= g (p ascending, p[0] = 0)
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (p[m] <= g) lo = m; else hi = m;
    }
    return lo;
}

// ranker report bits (CallCtl pad[5])
constexpr uint32_t LF_TIES = 1u;      // equal sums among the first pops + 1
constexpr uint32_t LF_VIOL = 2u;      // a fast-path condition failed for a tied or late line
constexpr uint32_t LF_FALLBACK = 4u;  // the rankers could not order this call at all
constexpr uint32_t LF_RANKED = 8u;    // a regime-B call the rankers took

#ifndef STG_FILL_STAMPS
#define STG_FILL_STAMPS 0
#endif
// diagnostics (STG_FILL_STAMPS builds): a ranker's phase stamps, words 32..41 (its clock 28, 29);
// worker 0's, words 16..23
#define LF_WSTAMP(i)                                                                                 \
    do {                                                                                             \
        if (STG_FILL_STAMPS && wk == 0 && threadIdx.x == 0)                                          \
            A.dbg[16 + (i)] = (uint32_t)__builtin_amdgcn_s_memrealtime();                            \
    } while (0)
#ifndef STG_FILL_STAMPS_RK
#define STG_FILL_STAMPS_RK 0  // the ranker whose phases are stamped
#endif
#define LF_STAMP(i)                                                                                  \
    do {                                                                                             \
        if (STG_FILL_STAMPS && rk == STG_FILL_STAMPS_RK && threadIdx.x == 0)                         \
            A.dbg[32 + (i)] = (uint32_t)__builtin_amdgcn_s_memrealtime();                            \
    } while (0)

// What every lfin workgroup decides, identically.
struct LfinDec {
    uint32_t Qtot, Wtot, kb, r, lim, c0, ct, cnt, M, N;
    bool regimeB, tail_cand, listw, lists_ok, any_big;  // any_big: a chunk lists more than LF_SPEC lines
    float t, inc, tail_key;
};

// Per-chunk counts -> exclusive prefixes in LDS, and the regime decision of
// tv16.hip finish_chunk (thresholdv16.cpp:138-259).
__device__ __forceinline__ void lfin_prefix(LfinLds &L, const LfinArgs &A, LfinDec &D) {
    const Tv16FillBucket &d = A.d;
    const uint32_t tid = threadIdx.x, nc = A.nc;
    constexpr uint32_t PER = LMAXC / FILL_WG;
    static_assert(PER * FILL_WG == LMAXC, "chunks per thread");
    // the ragged tail's floats, loaded with the counts (one round trip)
    float tv[16];
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i) tv[i] = i < d.tl ? d.src[(size_t)d.nb * 16 + i] : 0.f;
    uint32_t qv[PER], wv[PER], sq = 0, sw = 0, bad = 0, big = 0;
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) {
        const uint32_t c = tid * PER + u;
        const uint2 x = c < nc ? A.ldesc[c] : make_uint2(0u, 0u);  // {qualifying:16 | window:16, call tag}
        qv[u] = x.x & 0xffffu;
        wv[u] = x.x >> 16;
    }
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) {
        sq += qv[u];
        sw += wv[u];
        bad |= (qv[u] > LQCAP || wv[u] > LWCAP) ? 1u : 0u;
        big |= qv[u] > 16u ? 1u : 0u;
    }
    D.t = A.cp->t;
    D.inc = A.cp->inc;
    uint32_t pq = blk_excl_scan<FNW_F>(sq, L.sh, &D.Qtot);
    uint32_t pw = blk_excl_scan<FNW_F>(sw, L.sh, &D.Wtot);
#pragma unroll
    for (uint32_t u = 0; u < PER; ++u) {
        const uint32_t c = tid * PER + u;
        if (c < nc) { L.qp[c] = pq; L.wp[c] = pw; }
        pq += qv[u];
        pw += wv[u];
    }
    if (tid == 0) { L.qp[nc] = D.Qtot; L.wp[nc] = D.Wtot; }
    D.lists_ok = !__syncthreads_or((int)bad);
    D.any_big = __syncthreads_or((int)big);
    const uint32_t Qtot = D.Qtot;
    D.kb = d.dst_len / 16;
    D.r = d.dst_len % 16;
    D.lim = D.kb + (D.r ? 1u : 0u);
    D.c0 = Qtot >= D.lim ? d.dst_len : 16u * Qtot;
    D.tail_cand = false;
    D.tail_key = 0.f;
    D.ct = 0;
    if (D.c0 < d.dst_len && d.tl) {  // stage 3: the ragged tail's signed, sequential sum (thresholdv16.cpp:212-236)
        float sm = 0.f;
#pragma unroll
        for (uint32_t i = 0; i < 16; ++i)
            if (i < d.tl) sm += tv[i];
        if (sm * 16.0f >= D.t * (float)d.tl) D.ct = min(d.dst_len - D.c0, d.tl);
        else { D.tail_cand = true; D.tail_key = sm * 16.0f / (float)d.tl; }
    }
    D.cnt = D.c0 + D.ct;
    D.regimeB = D.cnt < d.dst_len;
    const uint32_t ncand = d.nb - Qtot;  // non-qualifying full lines
    D.M = D.regimeB ? min((d.dst_len - D.cnt + 15u) / 16u, ncand) : 0u;
    D.listw = D.regimeB && D.Wtot >= D.M && D.Wtot + 1 <= CAND_CAP;
    D.N = ncand + (D.tail_cand ? 1u : 0u);  // the reference's candidate vector length
}

// A chunk whose lists overflowed, read again from src by one workgroup, in
// order: its qualifying lines (emitted at their ranks) and window lines.
__device__ __forceinline__ void lfin_rescan(LfinLds &L, const Tv16FillBucket &d, uint32_t c, const LfinDec &D,
                                            bool emit, bool list) {
    const uint32_t tid = threadIdx.x;
    const uint32_t L0 = c * LCHUNK;
    const uint32_t nl = d.nb > L0 ? min(LCHUNK, d.nb - L0) : 0u;
    const uint32_t tb = f2u(D.t), wlo = tb > TV16_WIN ? tb - TV16_WIN : 0u;
    const bool vec = aligned16(d);
    uint32_t *cu = const_cast<uint32_t *>(d.cand), *cl = cu + CAND_CAP, *ci = cu + 2 * CAND_CAP;
    uint32_t qb = L.qp[c], wb = L.wp[c];
    for (uint32_t l0 = 0; l0 < nl; l0 += FILL_WG) {
        const uint32_t l = l0 + tid;
        const float sm = l < nl ? lane_line_sum(d.src + (size_t)(L0 + l) * 16) : 0.f;
        const uint32_t u = f2u(sm);
        const bool qf = l < nl && sm >= D.t;
        const bool wf = l < nl && u >= wlo && u < tb;
        uint32_t tq, tw;
        const uint32_t rq = blk_excl_scan<FNW_F>(qf ? 1u : 0u, L.sh, &tq);
        const uint32_t rw = blk_excl_scan<FNW_F>(wf ? 1u : 0u, L.sh, &tw);
        if (emit && qf && qb + rq < D.lim) {
            const uint32_t g = qb + rq;
            emit_line(d, vec, (L0 + l) * 16, 16 * g, g == D.kb ? D.r : 16u);
        }
        if (list && wf && wb + rw < CAND_CAP) {
            st_sc1(&cu[wb + rw], u);
            st_sc1(&cl[wb + rw], (L0 + l) * 16);
            st_sc1(&ci[wb + rw], L0 + l - (qb + rq));
        }
        qb += tq;
        wb += tw;
    }
}

// ---------------------------------------------------------------------------
// worker `wk`: the qualifying lines of its chunks, loaded with the counts
// ---------------------------------------------------------------------------
constexpr uint32_t LF_SPEC = 16;  // list slots per chunk loaded before the counts are known
__device__ __forceinline__ void lfin_store(const Tv16FillBucket &d, bool vec, uint32_t g, uint32_t kb, uint32_t r,
                                           uint32_t line, float4 x, uint32_t q) {
    const uint32_t len = g == kb ? r : 16u, off = 16 * g + 4 * q, pos = line * 16 + 4 * q;
    const uint32_t bi = pos + (uint32_t)d.idx_offset;
    if (vec && len == 16) {
        put_pair4(d, off, bi, x);
    } else {
        const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (uint32_t cc = 0; cc < 4; ++cc)
            if (4 * q + cc < len) {
                put_pair(d, off + cc, bi + cc, xs[cc]);
            }
    }
}

__device__ __noinline__ void lfin_worker(LfinLds &L, uint32_t wk) {
    const LfinArgs &A = L.args;
    const Tv16FillBucket &d = A.d;
    const uint32_t tid = threadIdx.x, nc = A.nc, nwk = A.workers;
    LF_WSTAMP(0);
    // ---- its chunks' first LF_SPEC listed lines (position, data), in flight
    //      with the counts: a lane per quarter line ----
    const uint32_t pc = (nc + nwk - 1) / nwk, c_lo = min(nc, wk * pc), c_hi = min(nc, c_lo + pc);
    constexpr uint32_t NS = 4;  // speculative quarter lines per thread
    const uint32_t nspec = min((c_hi - c_lo) * LF_SPEC * 4, NS * FILL_WG);
    uint32_t ls[NS];
    float4 xs[NS];
#pragma unroll
    for (uint32_t i = 0; i < NS; ++i) {
        const uint32_t t = tid + i * FILL_WG, c = c_lo + t / (LF_SPEC * 4), sl = (t / 4) % LF_SPEC;
        if (t < nspec) {
            ls[i] = A.lq[(size_t)c * LQCAP + sl] & 0xffffu;  // (the call's tag above the line)
            xs[i] = A.lv[((size_t)c * LQCAP + sl) * 4 + (t & 3u)];
        }
    }
    LfinDec D;
    lfin_prefix(L, A, D);
    LF_WSTAMP(1);
    const uint32_t *qp = L.qp;
    const bool vec = aligned16(d);
#pragma unroll
    for (uint32_t i = 0; i < NS; ++i) {
        const uint32_t t = tid + i * FILL_WG, c = c_lo + t / (LF_SPEC * 4), sl = (t / 4) % LF_SPEC;
        if (t >= nspec) continue;
        const uint32_t qc = qp[c + 1] - qp[c], g = qp[c] + sl;
        if (qc <= LQCAP && sl < qc && g < D.lim) lfin_store(d, vec, g, D.kb, D.r, c * LCHUNK + ls[i], xs[i], t & 3u);
    }
    LF_WSTAMP(2);
    // ---- the rest: slots past the speculative ones (chunks with more listed
    //      lines, or more chunks than the speculation covered) ----
    static_assert(LF_SPEC == 16, "lfin_prefix flags chunks with more than 16 listed lines");
    const uint32_t covered = nspec / (LF_SPEC * 4);  // chunks whose first LF_SPEC slots were taken
    for (uint32_t c = c_lo + (D.any_big ? 0u : covered); c < c_hi; ++c) {
        const uint32_t qc = qp[c + 1] - qp[c], s0 = c - c_lo < covered ? LF_SPEC : 0u;
        if (qc > LQCAP || qc <= s0 || qp[c] + s0 >= D.lim) continue;  // overflowed (re-read below), or done
        for (uint32_t t = s0 * 4 + tid; t < qc * 4; t += FILL_WG) {
            const uint32_t sl = t / 4, g = qp[c] + sl;
            if (g >= D.lim) continue;
            lfin_store(d, vec, g, D.kb, D.r, c * LCHUNK + (A.lq[(size_t)c * LQCAP + sl] & 0xffffu),
                       A.lv[((size_t)c * LQCAP + sl) * 4 + (t & 3u)], t & 3u);
        }
    }
    LF_WSTAMP(3);
    // ---- its chunks whose lists overflowed: read again ----
    if (!D.lists_ok) {
        for (uint32_t c = c_lo; c < c_hi; ++c) {
            const uint32_t qc = qp[c + 1] - qp[c];
            if (qc > LQCAP && qp[c] < D.lim) lfin_rescan(L, d, c, D, true, false);
        }
    }
    LF_WSTAMP(4);
    // ---- worker 0: tail, AIMD state, count, decision (tv16.hip finish_chunk) ----
    if (wk == 0 && tid == 0) {
        if (D.ct) {
            const size_t p0 = (size_t)d.nb * 16;
            for (uint32_t i = 0; i < D.ct; ++i) {
                put_pair(d, D.c0 + i, (uint32_t)(p0 + i) + (uint32_t)d.idx_offset, d.src[p0 + i]);
            }
        }
        if (A.resid && d.tl)  // fused error feedback: the ragged tail is not streamed
            for (uint32_t i = 0; i < d.tl; ++i) A.resid[(size_t)d.nb * 16 + i] = d.src[(size_t)d.nb * 16 + i];
        A.state->t = D.regimeB ? (float)((double)D.t * 0.99) : D.t + D.inc;  // thresholdv16.cpp:243-259
        A.state->inc = D.inc;
        A.state->init = 1;
        st_sc1(d.count_out, (uint32_t)min((uint64_t)d.dst_len, (uint64_t)d.nb * 16 + d.tl));
        if (ld_sc1(A.fail)) st_sc1(d.count_out, POISON_COUNT);
        uint32_t flags = 0;
        if (D.regimeB) flags = TV16_DEC_B | (D.tail_cand ? TV16_DEC_TAIL : 0u) | (D.listw ? TV16_DEC_WIN : 0u);
        Decision &Dc = A.dec[0];
        st_sc1(&Dc.w[1], ((uint64_t)D.cnt << 32) | D.M);
        st_sc1(&Dc.w[2], ((uint64_t)D.Wtot << 32) | __float_as_uint(D.tail_key));
        st_sc1(&Dc.w[3], ((uint64_t)D.Qtot << 32) | __float_as_uint(D.t));
        vm_drain();
        st_sc1(&Dc.w[0], ((uint64_t)((A.epoch << 8) | TV16_TAG_DEC) << 32) | flags);
    }
    LF_WSTAMP(5);
}

// The exact orderer's input, by the last workgroup when it has to order the
// fill itself: the window list in scan order (sum bits, position, candidate
// index), from the scan's lists or, for a chunk whose lists overflowed, from src.
__device__ __noinline__ void lfin_list(LfinLds &L) {
    const LfinArgs &A = L.args;
    const Tv16FillBucket &d = A.d;
    const uint32_t tid = threadIdx.x, nc = A.nc;
    LfinDec D;
    lfin_prefix(L, A, D);
    if (!D.listw) return;
    uint32_t *cu = const_cast<uint32_t *>(d.cand), *cl = cu + CAND_CAP, *ci = cu + 2 * CAND_CAP;
    const uint32_t *qp = L.qp, *wp = L.wp;
    for (uint32_t p = tid; p < nc * LWCAP; p += FILL_WG) {
        const uint32_t c = p / LWCAP, i = p % LWCAP;
        const uint32_t wc = wp[c + 1] - wp[c];
        if (i >= wc || wc > LWCAP || qp[c + 1] - qp[c] > LQCAP) continue;  // overflowed: re-read below
        const uint2 x = A.lw[(size_t)c * LWCAP + i];
        const uint32_t line = c * LCHUNK + (x.y & 0xffffu), e = wp[c] + i;
        st_sc1(&cu[e], x.x);
        st_sc1(&cl[e], line * 16);
        st_sc1(&ci[e], line - (qp[c] + (x.y >> 16)));
    }
    if (!D.lists_ok)
        for (uint32_t c = 0; c < nc; ++c) {
            const uint32_t qc = qp[c + 1] - qp[c], wc = wp[c + 1] - wp[c];
            if (wc && (wc > LWCAP || qc > LQCAP)) lfin_rescan(L, d, c, D, false, true);
        }
    vm_drain();
    __syncthreads();
}

// ---------------------------------------------------------------------------
// ranker `rk`: the regime-B fill's order for a share of the kept lines
// ---------------------------------------------------------------------------

__device__ __noinline__ void lfin_ranker(LfinLds &L, uint32_t rk) {
    const LfinArgs &A = L.args;
    const Tv16FillBucket &d = A.d;
    const uint32_t tid = threadIdx.x;
    LfinDec D;
    LF_STAMP(0);
    if (STG_FILL_STAMPS && rk == 0 && tid == 0) A.dbg[28] = (uint32_t)__builtin_amdgcn_s_memtime();  // the shader clock
    constexpr uint32_t PB = NBIN / FILL_WG;  // bins per thread
    static_assert(PB == 2 && NBIN == LNBIN, "two bins per thread");
    uint32_t h[PB];  // the scan's window entries per bin, in flight with the prefix's loads
#pragma unroll
    for (uint32_t u = 0; u < PB; ++u) h[u] = A.whist[whist_word(PB * tid + u)];
    lfin_prefix(L, A, D);
    LF_STAMP(1);
    if (!D.regimeB || (!D.M && !D.tail_cand)) return;  // nothing to fill
    auto give_up = [&]() {
        if (rk == 0 && threadIdx.x == 0) g_or(&A.cc->pad[5], LF_FALLBACK);
    };
    if (rk == 0 && tid == 0) g_or(&A.cc->pad[5], LF_RANKED);
    const uint32_t tb = f2u(D.t), wlo = tb > TV16_WIN ? tb - TV16_WIN : 0u;
    const bool tail_in = D.tail_cand && D.tail_key >= u2f(wlo);
    const uint32_t W = D.Wtot + (tail_in ? 1u : 0u);
    // a -0.0 tail ties +0.0 sums in the reference's float compare, not in ford() order
    if (!D.listw || !D.lists_ok || D.N > POS_LIM || W == 0 || A.mode ||
        (tail_in && (f2u(D.tail_key) & 0x80000000u))) {
        give_up();
        return;
    }
    // the tail's window offset and bin, as the scan bins a sum (a tail key
    // rounded up to t would sort above the window: the orderer takes it)
    if (tail_in && !(D.tail_key < D.t)) {
        give_up();
        return;
    }
    const uint32_t tw = tail_in ? tb - 1u - f2u(D.tail_key) : 0u, tbin = tail_in ? tw >> 8 : NONE;
    // ---- bin starts; keep the first bins holding M + 2 entries: every pop,
    //      the first line past them and its ties (a bin never splits equal sums) ----
    const uint32_t need = D.M + 2;
    {
        const uint32_t b0 = PB * tid, c0 = h[0] + (b0 == tbin ? 1u : 0u), c1 = h[1] + (b0 + 1 == tbin ? 1u : 0u);
        uint32_t tot;
        const uint32_t run = blk_excl_scan<FNW_F>(c0 + c1, L.sh, &tot);
        L.bin[b0] = run;
        L.bin[b0 + 1] = run + c0;
        if (run < need && run + c0 >= need) { L.cut = b0 + 1; L.wk = run + c0; }
        else if (run + c0 < need && run + c0 + c1 >= need) { L.cut = b0 + 2; L.wk = run + c0 + c1; }
        if (tid == 0) {
            L.bin[NBIN] = tot;
            if (tot < need) { L.cut = NBIN; L.wk = tot; }
            L.tail_rank = NONE;
            L.nlate = 0;
        }
        __syncthreads();
    }
    const uint32_t cut = L.cut, Wk = L.wk;
    const uint32_t rem = d.dst_len - D.cnt;
    // a kept bin with more entries than the scan could store, or too many kept
    const bool over = (PB * tid < cut && h[0] > LBCAP) || (PB * tid + 1 < cut && h[1] > LBCAP);
    if (__syncthreads_or((int)over) || Wk > EMAX || Wk == 0 || 16u * Wk < rem) {
        give_up();
        return;
    }
    LF_STAMP(2);
    uint64_t *const kg = L.u.r.kg;
    uint32_t *const kc = L.u.r.kc, *const kl = L.u.r.kl;
    uint16_t *const emap = L.u.r.emap, *const ord = L.u.r.ord;
    uint8_t *const tf = L.u.r.tf;
#pragma unroll
    for (uint32_t u = 0; u < PB; ++u) {
        const uint32_t b = PB * tid + u;
        if (b < cut)
            for (uint32_t e = L.bin[b]; e < L.bin[b + 1]; ++e) emap[e] = (uint16_t)b;
    }
    __syncthreads();
    // ---- the kept entries, loaded together, decoded into LDS ----
    constexpr uint32_t KE = EMAX / FILL_WG;
    auto is_tail = [&](uint32_t e, uint32_t b) { return b == tbin && e + 1 == L.bin[b + 1]; };  // its bin's last
    {
        uint2 x[KE];
#pragma unroll
        for (uint32_t j = 0; j < KE; ++j) {
            const uint32_t e = tid + j * FILL_WG;
            x[j] = make_uint2(0u, 0u);
            if (e < Wk) {
                const uint32_t b = emap[e];
                if (!is_tail(e, b)) x[j] = A.went[b * LBCAP + (e - L.bin[b])];
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < KE; ++j) {
            const uint32_t e = tid + j * FILL_WG;
            if (e >= Wk) continue;
            uint32_t w, cx, line;
            if (is_tail(e, emap[e])) {  // the candidate vector's last entry (thresholdv16.cpp:229-234)
                w = tw;
                cx = D.N - 1;
                line = d.nb;
            } else {
                const uint32_t c = x[j].y >> 19;
                line = c * LCHUNK + ((x[j].y >> 10) & 511u);
                w = tb - 1u - x[j].x;
                cx = line - (L.qp[c] + (x[j].y & 1023u));
            }
            kg[e] = (uint64_t)w << 25 | rf_key(cx);
            kc[e] = cx;
            kl[e] = line;
        }
    }
    __syncthreads();
    LF_STAMP(3);
    // ---- ranks: (sum desc = window offset asc, right-first pre-order of the
    //      start position asc) = kg asc; the bins are ordered, so an entry's
    //      rank is its bin's start plus the bin's smaller keys.  Ties (equal
    //      offsets) are noted for the fast path's check (3) ----
    for (uint32_t e = tid; e < Wk; e += FILL_WG) {
        const uint32_t b = emap[e], lo = L.bin[b], hi = L.bin[b + 1];
        const uint64_t ge = kg[e];
        const uint32_t we = (uint32_t)(ge >> 25);
        uint32_t r = lo;
        bool tie = false;
        for (uint32_t x = lo; x < hi; ++x) {
            const uint64_t gx = kg[x];
            r += gx < ge;
            tie |= (uint32_t)(gx >> 25) == we && gx != ge;
        }
        uint32_t f = 0;
        if (tie) {  // rare: is a tied line's start below this one's?
            f = LF_TIES;
            const uint32_t qe = kc[e] + 1;
            for (uint32_t x = lo; x < hi; ++x)
                if (x != e && (uint32_t)(kg[x] >> 25) == we && is_desc(kc[x] + 1, qe)) f |= LF_VIOL;
        }
        tf[e] = (uint8_t)f;
        ord[r] = (uint16_t)e;
        if (is_tail(e, b)) L.tail_rank = r;
    }
    __syncthreads();
    LF_STAMP(4);
    // ---- the pops P and the bound Ph of tv16fill.hip; R = keys >= the key at rank Ph ----
    const uint32_t tr = L.tail_rank;
    if (tr != NONE && 16u * Wk - (16u - d.tl) < rem) {
        give_up();
        return;
    }
    uint32_t P = (rem + 15u) / 16u;  // the first rank whose output offset reaches rem
    if (tr < P) P = (rem + (16u - d.tl) + 15u) / 16u;
    P = min(P, Wk);
    // conservative bounds for the fast-path conditions: one more pop than P
    // (the exact orderer counts its pops in (sum desc, index asc) order)
    const uint32_t Ph = min(P + 1, Wk - 1);
    const uint32_t late = D.N > Ph + 1 ? D.N - (Ph + 1) : 0u;  // start positions >= late: the last Ph + 1
    // ---- this ranker's share of the pops: four lanes per line, the loads of
    //      NRD rounds in flight (issued now, stored after the checks) ----
    const uint32_t nr = A.rankers, per = (P + nr - 1) / nr;
    const uint32_t s0 = min(P, rk * per), s1 = min(P, s0 + per);
    const bool vec = aligned16(d) && (D.cnt & 3u) == 0;
    auto offset = [&](uint32_t i) { return 16u * i - (tr < i ? 16u - d.tl : 0u); };
    constexpr uint32_t LPR = FILL_WG / 4, NRD = 4;
    const uint32_t q = tid & 3u;
    float4 v0, v1, v2, v3;
    uint32_t pos[NRD], off[NRD], len[NRD];
#define LF_LOAD_ROUND(J0)                                                                   \
    do {                                                                                    \
        _Pragma("unroll") for (uint32_t u = 0; u < NRD; ++u) {                              \
            const uint32_t i = (J0) + u * LPR + (tid >> 2);                                 \
            len[u] = 0;                                                                     \
            if (i < s1) {                                                                   \
                off[u] = offset(i);                                                         \
                if (off[u] < rem) {                                                         \
                    len[u] = min(i == tr ? d.tl : 16u, rem - off[u]);                       \
                    pos[u] = kl[ord[i]] * 16;                                               \
                }                                                                           \
            }                                                                               \
        }                                                                                   \
        auto ld4 = [&](uint32_t u) {                                                        \
            return (vec && len[u] == 16 && (off[u] & 3u) == 0)                              \
                       ? reinterpret_cast<const float4 *>(d.src + pos[u])[q]                \
                       : make_float4(0.f, 0.f, 0.f, 0.f);                                   \
        };                                                                                  \
        v0 = ld4(0); v1 = ld4(1); v2 = ld4(2); v3 = ld4(3);                                 \
    } while (0)
    auto store1 = [&](uint32_t u, float4 x) {
        if (!len[u]) return;
        const uint32_t o = D.cnt + off[u] + 4 * q, bi = pos[u] + 4 * q + (uint32_t)d.idx_offset;
        if (vec && len[u] == 16 && (off[u] & 3u) == 0) {
            put_pair4(d, o, bi, x);
        } else {
            for (uint32_t cc = 0; cc < 4; ++cc)
                if (4 * q + cc < len[u]) {
                    put_pair(d, o + cc, bi + cc, d.src[(size_t)pos[u] + 4 * q + cc]);
                }
        }
    };
    LF_LOAD_ROUND(s0);
    // ---- the fast path's conditions (tv16fill.hip (3)) for R; every ranker
    //      finds the same, ranker 0 reports ----
    const uint32_t wh = (uint32_t)(kg[ord[Ph]] >> 25);  // R: window offsets <= wh
    uint32_t fl = 0;
    for (uint32_t e = tid; e < Wk; e += FILL_WG) {
        if ((uint32_t)(kg[e] >> 25) > wh) continue;
        fl |= tf[e];
        const uint32_t ce = kc[e];
        if (ce >= late && ce) {  // a late line of R
            const uint32_t i = atomicAdd(&L.nlate, 1u);
            if (i < 64) L.late[i] = ce;
        }
    }
    __syncthreads();
    {   // no line of R at a late line's parent or sibling
        const uint32_t nl = L.nlate;
        if (nl > 64) fl |= LF_VIOL;
        else if (nl)
            for (uint32_t f = tid; f < Wk; f += FILL_WG) {
                if ((uint32_t)(kg[f] >> 25) > wh) continue;
                const uint32_t cf = kc[f];
                for (uint32_t i = 0; i < nl; ++i) {
                    const uint32_t ce = L.late[i];
                    if (cf == (ce - 1) / 2 || cf == ((ce - 1) ^ 1u) + 1) fl |= LF_VIOL;
                }
            }
    }
    LF_STAMP(5);
    store1(0, v0); store1(1, v1); store1(2, v2); store1(3, v3);
    for (uint32_t j0 = s0 + NRD * LPR; j0 < s1; j0 += NRD * LPR) {
        LF_LOAD_ROUND(j0);
        store1(0, v0); store1(1, v1); store1(2, v2); store1(3, v3);
    }
#undef LF_LOAD_ROUND
    const bool ties = __syncthreads_or((int)(fl & LF_TIES));
    const bool viol = __syncthreads_or((int)(fl & LF_VIOL));
    if (rk == 0 && tid == 0 && (viol || ties)) g_or(&A.cc->pad[5], (ties ? LF_TIES : 0u) | (viol ? LF_VIOL : 0u));
    if (STG_FILL_STAMPS && rk == STG_FILL_STAMPS_RK && tid == 0) { A.dbg[44] = Wk; A.dbg[45] = P; A.dbg[46] = s1 - s0; A.dbg[47] = fl; }
    LF_STAMP(6);
    LF_STAMP(7);
    LF_STAMP(8);
    LF_STAMP(9);
    if (STG_FILL_STAMPS && rk == 0 && tid == 0) A.dbg[29] = (uint32_t)__builtin_amdgcn_s_memtime();
}
