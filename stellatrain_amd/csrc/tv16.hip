// tv16.hip -- thresholdv16 ("cache-aware" threshold-v) on gfx950: the scan.
//
// Reference: ThresholdvCompressor16::impl_simd_v2
// (/root/reference/backend/src/compress/thresholdv16.cpp:78-295), first
// threshold impl_get_first_threshold (:36-54), line sum hsum_float_avx (:57-73).
//
// Semantics: walk 16-float lines in index order; a line whose
// tree-ordered |x| sum S >= t is emitted whole while >= 16 slots remain
// (stage 1); with r = dst_len % 16 slots left the next qualifying line donates
// its first r elements (stage 2); a ragged tail is judged on its *signed* sum
// (stage 3); if the scan ran dry the rest is filled from the non-qualifying
// lines in libstdc++ priority_queue order (heap fill, tv16fill.hip).  AIMD:
// t *= 0.99 (in double) when the scan ran dry, t += inc otherwise.
//
// One persistent launch per batch of buckets (tv16_batch).  The buckets are
// cut into 2048-line chunks (128 KiB), taken in order by 768-thread
// workgroups (two per CU) from a per-call counter -- every slot, the first two included --
// so fast workgroups take more chunks and every wait below points at a chunk
// an already-running workgroup has taken: the launch needs no workgroup to be
// co-resident with any other.  The 12 waves of a workgroup are specialised:
//
//   streaming waves  scan chunk after chunk and never wait on another
//             workgroup: stream the chunk once (a quad of lanes per line, DPP
//             cross-lane adds in the AVX tree order), stage the qualifying
//             lines' data in LDS with one ballot per 16-line step (their
//             in-chunk order), list the lines in a window just below t, and
//             count both; the last wave done with a chunk publishes its
//             aggregate counts.  They stall only when NBUF chunks ahead of
//             the finisher (LDS buffer sets in use).
//   finisher wave  per chunk: decoupled look-back over the bucket's earlier
//             chunks for the prefix counts, emit the chunk's qualifying lines
//             with rank < kb (+1 partial) straight from LDS, write its window
//             list (line sum, position, index in the reference's candidate
//             vector) at its window offset; the bucket's last chunk decides
//             the regime and writes the tail, the AIMD threshold, the count
//             and the decision.
//
// The regime-B heap fill runs in the follow-on launch tv16_fill (same stream,
// one workgroup per bucket), which reproduces libstdc++'s pop order exactly.
// A key's first call runs tv16_seq_sums + a radix select (select.hip) before
// the launch.
#include <algorithm>
#include <cstdlib>

#include "tv16_dev.h"

namespace stg {

namespace {

using namespace tv16;
constexpr uint32_t kEfAux = 2;  // cache policy of the fused residual stores (2: nontemporal)

constexpr uint32_t kTv16Ns = 11;
constexpr uint32_t FWG = (kTv16Ns + 1) * 64;  // workgroup: the streaming waves + the finisher
constexpr uint32_t FNW = FWG / 64;
constexpr uint32_t NS = kTv16Ns;  // streaming waves 0..NS-1
constexpr uint32_t FIN = NS;          // the finisher; waves past it (if any) idle
static_assert(NS + 1 <= FNW && FWG <= 1024, "streaming group + finisher fit the workgroup");
constexpr uint32_t kTv16Nbuf = 5;
constexpr uint32_t kTv16ScanD = 3;
constexpr uint32_t NBUF = kTv16Nbuf;  // LDS buffer sets (slots) in flight per workgroup
constexpr uint32_t CIDR = 2 * NBUF;       // chunk-id ring
constexpr uint32_t kTv16StageB = 72;
constexpr uint32_t kTv16WlB = 64;
constexpr uint32_t STAGE_B = kTv16StageB;  // qualifying lines staged in LDS per slot (~20 expected at 1%)
constexpr uint32_t WL_B = kTv16WlB;  // window candidates listed in LDS per slot
constexpr uint32_t kTv16PollSleep = 8;  // s_sleep units (64 clocks) between prefix polls
constexpr uint32_t GB = 512;        // chunk descriptors gathered per round trip (a 64 MiB bucket has 512)
// float4 loads in flight per streaming wave: 2 x 14 x 64 x 16 B x SCAN_D per CU
// (SCAN_D = 3: 84 KiB per CU, just over the ~72 KiB that hides an HBM miss;
// deeper queues add latency to every exchange round trip -- Little's law)
constexpr uint32_t SCAN_D_BATCH = kTv16ScanD;
// A one-bucket launch (its fill runs after it, nothing else of the codec
// beside it): each workgroup streams one chunk, so twice the loads in flight
// halve its round trips; 6 waves per SIMD leave it ~80 VGPRs.
constexpr uint32_t kTv16ScanDLone = 6;
constexpr uint32_t SCAN_D_LONE = kTv16ScanDLone;
constexpr uint32_t MAXG = 512;      // workgroups per launch (2 per CU)
// ---------------------------------------------------------------------------
// first call: sequential |x| sums per line, last partial line scaled by
// 16/(n%16) (thresholdv16.cpp:44-50)
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(STG_WG) tv16_seq_sums(const float *__restrict__ src, size_t n,
                                                        float *__restrict__ out, uint32_t nblk) {
    const uint32_t j = blockIdx.x * STG_WG + threadIdx.x;
    if (j >= nblk) return;
    const size_t base = (size_t)j * 16;
    const uint32_t len = (uint32_t)std::min<size_t>(16, n - base);
    float s = 0.f;
    if (len == 16) {
        const float4 *p = reinterpret_cast<const float4 *>(src + base);
        const float4 a = p[0], b = p[1], c = p[2], d = p[3];
        s += fabsf(a.x); s += fabsf(a.y); s += fabsf(a.z); s += fabsf(a.w);
        s += fabsf(b.x); s += fabsf(b.y); s += fabsf(b.z); s += fabsf(b.w);
        s += fabsf(c.x); s += fabsf(c.y); s += fabsf(c.z); s += fabsf(c.w);
        s += fabsf(d.x); s += fabsf(d.y); s += fabsf(d.z); s += fabsf(d.w);
    } else {
        for (uint32_t i = 0; i < len; ++i) s += fabsf(src[base + i]);
        s *= 16.0f / (float)len;
    }
    out[j] = s;
}

__global__ void tv16_init_state(KeyState *st, const RSel *rs) {
    const float t = u2f(rs->prefix);
    st->t = t;
    st->inc = (float)((double)t * 0.01);
    st->init = 1;
}

// ---------------------------------------------------------------------------
// batched persistent kernel
// ---------------------------------------------------------------------------
struct BucketDesc {  // 88 bytes
    const float *src;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    float *sums_g;    // unused by the scan (first-threshold sums, the fill's heap)
    uint32_t nb, tl, dst_len;
    int32_t idx_offset;
    uint32_t cs, nc;  // chunks [cs, cs + nc) of the launch's chunk sequence (nc >= 1)
    float *resid;     // fused error feedback: the streaming waves copy every full line here (or null)
    uint32_t wflag, wend;  // wire form of the emitted pairs (wire_dev.h; 0: u32 / f32)
};

struct BatchArgs {
    BucketDesc bk[MAX_BATCH];
    uint32_t nbk;
    uint32_t epoch;  // 1 .. 2^24-1
    uint32_t K;      // chunks in the launch
    FillCtl *ctl;
    ChunkDesc *desc;
    uint32_t *cand;
    uint32_t *fail;
};

// LDS of one workgroup (< 80 KiB: two workgroups per CU).
struct Lds {
    // streaming waves -> finisher, by buffer set (slot % NBUF)
    float4 stage[NBUF][STAGE_B * 4];     // staged qualifying lines (64 B each)
    uint32_t stage_line[NBUF][STAGE_B];
    uint64_t wl[NBUF][WL_B];             // window candidates: line-sum bits << 32 | element position
    uint32_t nst[NBUF];                  // qualifying lines staged (slot counter)
    uint32_t nwl[NBUF];                  // window candidates listed (slot counter)
    uint32_t qcnt[NBUF];                 // qualifying lines of the chunk
    uint32_t wcnt[NBUF];                 // window lines of the chunk
    uint32_t sdone[NBUF];                // streaming waves done with the chunk
    float tval[NBUF], incv[NBUF];        // the bucket's threshold state as scanned
    uint32_t cid[CIDR];                  // chunk of slot j at [j % CIDR] (>= K: no more chunks)
    uint32_t cok[CIDR];                  // j + 1 once cid[j % CIDR] holds slot j's chunk
    uint32_t mid[CIDR];                  // waves past the middle of slot j (j % CIDR)
    uint32_t fdone;                      // slots released by the finisher
    // finisher
    uint4 gb[GB];                        // gathered chunk descriptors (one piece of a bucket)
};
static_assert(sizeof(Lds) <= TV16_SCAN_LDS, "two scan workgroups and a fill workgroup share a CU");

// Spin-timeout failure bits: FAIL_SPIN_TIMEOUT plus bit 8 + site naming the
// wait that gave up: 1 buffer set, 2 prefix aggregates, 3 chunk streamed,
// 6 / 7 slot chunk id (streamer / finisher).
__device__ __forceinline__ constexpr uint32_t spin_site(uint32_t site) { return FAIL_SPIN_TIMEOUT | (1u << (8 + site)); }

struct Ctx {
    const BatchArgs &A;
    Lds &L;
    uint32_t G, w;
    FillCtl *ctlp;
    uint32_t *candp;
    uint32_t *failp;

    __device__ __forceinline__ uint32_t tag(uint32_t kind) const { return (A.epoch << 8) | kind; }
    __device__ __forceinline__ FillCtl *ctl() const { return ctlp; }
    __device__ __forceinline__ CallCtl *cc() const { return &ctlp->cc[A.epoch & 1u]; }
    __device__ __forceinline__ uint32_t *cand(uint32_t b) const { return candp + (size_t)b * CAND_WORDS; }
    __device__ __forceinline__ void fail(uint32_t bits) const { g_or(failp, bits); }
    // A spin timeout: its site bit, and for the first one in the workspace's
    // life a record for the host's error message: {site + 1, workgroup, x0,
    // x1, x2, epoch} at fail[1..6]; per site, its first one at fail[8 + 4 site].
    // Every bucket's count is poisoned: the launch's output cannot be trusted.
    __device__ __forceinline__ void spin_fail(uint32_t site, uint32_t x0, uint32_t x1, uint32_t x2) const {
        g_or(failp, spin_site(site));
        if (atomicCAS(failp + 1, 0u, site + 1u) == 0u) {
            st_sc1(failp + 2, w);
            st_sc1(failp + 3, x0);
            st_sc1(failp + 4, x1);
            st_sc1(failp + 5, x2);
            st_sc1(failp + 6, A.epoch);
        }
        uint32_t *rec = failp + 8 + 4 * site;  // and each site's first one: {workgroup + 1, x0, x1, x2}
        if (atomicCAS(rec, 0u, w + 1u) == 0u) {
            st_sc1(rec + 1, x0);
            st_sc1(rec + 2, x1);
            st_sc1(rec + 3, x2);
        }
        for (uint32_t b = 0; b < A.nbk; ++b) st_sc1(A.bk[b].count_out, POISON_COUNT);
    }
    // bucket holding global chunk k (scalar search over <= 16 buckets)
    __device__ __forceinline__ uint32_t bucket_of(uint32_t k) const {
        uint32_t b = 0;
        while (b + 1 < A.nbk && k >= A.bk[b + 1].cs) ++b;
        return b;
    }
};

constexpr uint32_t TAG_AGG = 1, TAG_DEC = TV16_TAG_DEC;
constexpr uint32_t DEC_B = TV16_DEC_B, DEC_WIN = TV16_DEC_WIN, DEC_TAIL = TV16_DEC_TAIL;
constexpr uint32_t WIN = TV16_WIN;

// ===========================================================================
// streaming waves
// ===========================================================================
// scan of slot j = chunk k by streaming wave s: lines i = (s + NS*m)*16 +
// lane/4 of the chunk, m = 0, 1, ...; SCAN_D float4 loads per lane in flight
// through a buffer descriptor bounded to the chunk (lanes past it read zeros).
template <int STAGE, bool EF, uint32_t SCAN_D>
__device__ __forceinline__ void scan_chunk(Ctx &C, uint32_t j, uint32_t k, uint32_t s) {
    Lds &L = C.L;
    const uint32_t par = j % NBUF;
    if (j >= NBUF) {  // buffer set `par` is free once the finisher released slot j - NBUF
        uint64_t st2 = 0;
        uint32_t spins = 0;
        for (; lds_ld(&L.fdone) < j + 1 - NBUF; ++spins) {
            __builtin_amdgcn_s_sleep(2);
            if (spin_expired(spins, st2)) { if (flane() == 0) C.spin_fail(1, j, lds_ld(&L.fdone), s); break; }
        }
    }
    const uint32_t b = C.bucket_of(k);
    const BucketDesc &d = C.A.bk[b];
    const uint32_t c = k - d.cs;
    const uint32_t L0 = c * TV16_CHUNK;
    const uint32_t nl = d.nb > L0 ? std::min(TV16_CHUNK, d.nb - L0) : 0u;
    // Read before this chunk's counts are published: the bucket's last chunk
    // rewrites the state only after every chunk's counts are in.
    const float t = uni(d.state->t);
    const uint32_t lane = flane(), q = lane & 3;
    if (s == 0 && lane == 0) { L.tval[par] = t; L.incv[par] = uni(d.state->inc); }
    const uint32_t tb = f2u(t);
    const uint32_t wlo = tb > WIN ? tb - WIN : 0u;  // window [wlo, tb) just below t
    const uint32_t steps = (nl + 15) / 16;          // 16 lines per wave step
    const uint32_t mine = steps > s ? (steps - s + NS - 1) / NS : 0u;
    uint32_t cnt_w = 0, win_w = 0;
    // nontemporal buffer loads; the whole offset goes in voffset so the
    // hardware range check sees it
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(d.src + (size_t)L0 * 16), 0, nl * 64u, 0x00020000);
    const uint32_t lane_line = s * 16 + (lane >> 2);
    // fused error feedback (compress.cpp:185's memcpy(residual, src)): each
    // streamed granule is also stored, nontemporally, to the residual; the
    // selected entries are zeroed afterwards (ef_zero) as the reference does
    // (EF: a separate instantiation, so the plain codec carries none of it)
    const __amdgpu_buffer_rsrc_t rsrc_r = __builtin_amdgcn_make_buffer_rsrc(
        EF ? d.resid + (size_t)L0 * 16 : nullptr, 0, (EF && d.resid) ? nl * 64u : 0u, 0x00020000);
    auto store_r = [&](uint32_t m, float4 x) {
        uint32_t voff = lane_line * 64u + q * 16u;
        asm volatile("" : "+v"(voff));
        u4v t4;
        t4.x = __float_as_uint(x.x); t4.y = __float_as_uint(x.y); t4.z = __float_as_uint(x.z); t4.w = __float_as_uint(x.w);
        __builtin_amdgcn_raw_buffer_store_b128(t4, rsrc_r, voff + m * (NS * 1024u), 0, kEfAux /* 2 = nt */);
    };
    auto load = [&](uint32_t m) -> float4 {
        uint32_t voff = lane_line * 64u + q * 16u;
        asm volatile("" : "+v"(voff));  // opaque: no hoisted per-step offsets
        const u4v t4 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + m * (NS * 1024u), 0, 2 /* nt */);
        return make_float4(__uint_as_float(t4.x), __uint_as_float(t4.y), __uint_as_float(t4.z),
                           __uint_as_float(t4.w));
    };
    // rolling pipeline: step m + SCAN_D is issued as soon as step m is consumed
    float4 v[SCAN_D];
#pragma unroll
    for (uint32_t u = 0; u < SCAN_D; ++u) v[u] = load(u);
    // The first wave past the middle of slot j takes the chunk of slot j + 1
    // from the call's counter (slot 0 at the start): late enough that chunks
    // are taken close to when they are streamed (the finishers' prefix counts
    // wait on earlier chunks only) and that a short batch spreads one chunk
    // per workgroup, early enough that the round trip hides behind the second
    // half of the slot.  Every wave in slot j has seen slot j's chunk id, so a
    // workgroup's chunk ids increase slot by slot and the first id >= K ends
    // it with no chunk left behind.
    uint32_t nx = 0;
    bool grab = false, tried = false;
    auto try_take = [&]() {
        tried = true;
        uint32_t first = 1;
        if (flane() == 0) first = atomicAdd(&L.mid[j % CIDR], 1u);
        grab = uni(first) == 0;
        // a launch with no more chunks than workgroups hands every chunk out
        // at slot 0 (each workgroup takes one as it starts): the counter has
        // nothing left, so skip its round trip (and the traffic on its line)
        if (grab && flane() == 0) nx = C.A.K <= C.G ? C.A.K : g_add(&C.cc()->next, 1u);
    };
    for (uint32_t m0 = 0; m0 < mine; m0 += SCAN_D) {
        if (!tried && m0 >= mine / 2) try_take();
#pragma unroll
        for (uint32_t u = 0; u < SCAN_D; ++u) {
            const float4 x = v[u];
            uint32_t ll = lane_line;
            asm volatile("" : "+v"(ll));
            const uint32_t i = (m0 + u) * (NS * 16u) + ll;  // line within the chunk
            if (STAGE == 3) {
                cnt_w += f2u(x.x + x.y + x.z + x.w) == 0x7f800001u;
                v[u] = load(m0 + u + SCAN_D);
                continue;
            }
            const float S = quad_line_sum(x);  // the same in all four lanes of the quad
            if (EF) store_r(m0 + u, x);
            v[u] = load(m0 + u + SCAN_D);
            const uint32_t us = f2u(S);
            // one test for the common case: no line of the step reaches the
            // window [wlo, tb) or the threshold (sums are >= +0, so us >= tb
            // iff S >= t for every non-NaN S)
            const bool near = i < nl && us >= wlo;
            if (!__ballot(near && q == 0)) continue;
            const bool qual = near && S >= t;
            const bool win = near && us < tb;
            const uint64_t bq = __ballot(qual && q == 0);
            const uint64_t bw = __ballot(win && q == 0);
            if (bw) {  // list the window candidates (composite keys)
                win_w += (uint32_t)__popcll(bw);
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&L.nwl[par], (uint32_t)__popcll(bw));
                base = __builtin_amdgcn_readfirstlane(base);
                if (win && q == 0) {
                    const uint32_t slot = base + (uint32_t)__popcll(bw & below_mask(flane()));
                    if (slot < WL_B) L.wl[par][slot] = ((uint64_t)us << 32) | ((L0 + i) * 16);
                }
            }
            if (bq) {  // stage the qualifying lines (all four lanes of each quad)
                cnt_w += (uint32_t)__popcll(bq);
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&L.nst[par], (uint32_t)__popcll(bq));
                base = __builtin_amdgcn_readfirstlane(base);
                if (qual) {
                    // qualifying quads before this one: bq has bits only at quad
                    // leaders, so leader p < this leader iff p + 3 < lane
                    const uint64_t b3 = bq << 3;
                    const uint32_t slot = base + __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(b3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b3, 0u));
                    if (slot < STAGE_B) {
                        const uint32_t lq = flane() & 3u;
                        L.stage[par][slot * 4 + lq] = x;
                        if (lq == 0) L.stage_line[par][slot] = i;
                    }
                }
            }
        }
    }
    if (!tried) try_take();  // no steps here (a short chunk)
    if (grab && flane() == 0) {
        // slot j + NBUF reuses slot j - NBUF's counter: every wave is done
        // with slot j - NBUF (the finisher released it) and none is past j yet
        L.mid[(j + NBUF) % CIDR] = 0;
        L.cid[(j + 1) % CIDR] = nx;
        lds_drain();
        lds_st(&L.cok[(j + 1) % CIDR], j + 2);
    }
    if (lane == 0) {
        if (cnt_w) atomicAdd(&L.qcnt[par], cnt_w);
        if (win_w) atomicAdd(&L.wcnt[par], win_w);
    }
    lds_drain();
    uint32_t old = 0;
    if (lane == 0) old = atomicAdd(&L.sdone[par], 1u);
    if (STAGE != 1 && STAGE != 3 && uni(old) == NS - 1 && lane == 0) {
        // the last streaming wave of the chunk publishes its aggregate at once
        // (every other wave's count adds were drained before its sdone add)
        const uint32_t aq = std::min(lds_ld(&L.qcnt[par]), 0xffffu), aw = std::min(lds_ld(&L.wcnt[par]), 0xffffu);
        st_sc1(&C.A.desc[k].agg, ((uint64_t)C.tag(TAG_AGG) << 32) | (aq << 16) | aw);
    }
}

// ===========================================================================
// finisher wave
// ===========================================================================
__device__ __forceinline__ void release(Ctx &C, uint32_t par, uint32_t j) {
    Lds &L = C.L;
    lds_drain();
    if (flane() == 0) {
        L.nst[par] = 0;
        L.nwl[par] = 0;
        L.qcnt[par] = 0;
        L.wcnt[par] = 0;
        L.sdone[par] = 0;
    }
    lds_drain();
    if (flane() == 0) lds_st(&L.fdone, j + 1);
}

// Prefix counts of chunk c of bucket b: the aggregates of the bucket's chunks
// before c (tagged 16-byte descriptors, gathered GB per round trip into LDS;
// stale ones re-polled).  Chunks are taken in order, so these were taken
// earlier than chunk c and are almost always complete.  The bucket's last
// chunk thereby also sees every other chunk: its prefix + its own counts are
// the bucket's totals.
__device__ __forceinline__ void prefix_counts(Ctx &C, uint32_t b, uint32_t c, uint32_t &P, uint32_t &Wbef) {
    Lds &L = C.L;
    const BucketDesc &d = C.A.bk[b];
    const uint32_t lane = flane();
    const uint32_t tA = C.tag(TAG_AGG);
    uint32_t pq = 0, pw = 0;
    for (uint32_t p0 = 0; p0 < c; p0 += GB) {
        const uint32_t n = std::min(GB, c - p0);
        gather16(&C.A.desc[d.cs + p0], n, L.gb);
        for (uint32_t i0 = 0; i0 < n; i0 += 64) {
            const uint32_t i = i0 + lane;
            uint64_t a = 0;
            if (i < n) { const uint4 e = L.gb[i]; a = ((uint64_t)e.y << 32) | e.x; }
            bool pend = i < n && (uint32_t)(a >> 32) != tA;
            // Stale ones: poll only the latest pending chunk (taken last, so
            // almost always published last) from one lane, then re-read the
            // rest once -- every finisher polling every stale descriptor
            // floods the fabric the streaming loads share.
            uint64_t st4 = 0;
            for (uint32_t spins = 0;; ++spins) {
                const uint64_t pm = __ballot(pend);
                if (!pm) break;
                const uint32_t hl = 63u - (uint32_t)__clzll((long long)pm);
                __builtin_amdgcn_s_sleep(kTv16PollSleep);
                if (lane == hl) {
                    a = ld_sc1(&C.A.desc[d.cs + p0 + i].agg);
                    pend = (uint32_t)(a >> 32) != tA;
                }
                if (!__ballot(lane == hl && pend) && pend) {
                    a = ld_sc1(&C.A.desc[d.cs + p0 + i].agg);
                    pend = (uint32_t)(a >> 32) != tA;
                }
                if (spin_expired(spins, st4)) { {
                    const uint32_t pi = uni((uint32_t)__builtin_amdgcn_readlane((int)(p0 + i), (int)hl));
                    const uint32_t tg = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a >> 32), (int)hl);
                    if (lane == 0) C.spin_fail(2, c, pi, tg);
                    break;
                } }
            }
            if (i < n) { pq += (uint32_t)(a >> 16) & 0xffffu; pw += (uint32_t)a & 0xffffu; }
        }
    }
    P = uni(wave_sum(pq));
    Wbef = uni(wave_sum(pw));
}

// finish(slot j = chunk k): look-back, ordered emission, window list; the
// bucket's last chunk also decides the regime and writes tail / AIMD / count
// and the decision the fill launch reads.
template <int STAGE>
__device__ __forceinline__ void finish_chunk(Ctx &C, uint32_t j, uint32_t k) {
    Lds &L = C.L;
    const uint32_t par = j % NBUF;
    const uint32_t lane = flane();
    uint64_t st5 = 0;
    for (uint32_t spins = 0; lds_ld(&L.sdone[par]) < NS; ++spins) {
        __builtin_amdgcn_s_sleep(1);
        if (spin_expired(spins, st5)) { if (lane == 0) C.spin_fail(3, j, lds_ld(&L.sdone[par]), k); break; }
    }
    if (STAGE == 1 || STAGE == 3) {
        release(C, par, j);
        return;
    }
    const uint32_t b = C.bucket_of(k);
    const BucketDesc &d = C.A.bk[b];
    const uint32_t c = k - d.cs;
    const uint32_t L0 = c * TV16_CHUNK;
    const uint32_t nl = d.nb > L0 ? std::min(TV16_CHUNK, d.nb - L0) : 0u;
    const uint32_t qw = uni(L.qcnt[par]);
    const float t = uni(L.tval[par]), inc = uni(L.incv[par]);

    // ---- prefix counts of the bucket's earlier chunks ----
    uint32_t P = 0, Wbef = 0;
    if (c) prefix_counts(C, b, c, P, Wbef);
    const uint32_t ww = uni(L.wcnt[par]);

    // ---- ordered emission of the chunk's qualifying lines with rank < lim ----
    const uint32_t kb = d.dst_len / 16, r = d.dst_len % 16;
    const uint32_t lim = kb + (r ? 1u : 0u);
    const bool vec = aligned16(d);
    if (P < lim && qw) {
        if (qw <= STAGE_B) {
            // every qualifying line is staged in LDS with its line index: its
            // in-chunk rank is the number of staged lines before it; a quad
            // of lanes per line
            const uint32_t q = lane & 3;
            for (uint32_t e0 = 0; e0 < qw; e0 += 16) {
                const uint32_t e = e0 + (lane >> 2);
                if (e >= qw) continue;
                const uint32_t i = L.stage_line[par][e];
                uint32_t g = P;
                for (uint32_t x = 0; x < qw; ++x) g += L.stage_line[par][x] < i;
                if (g >= lim) continue;
                const uint32_t pos = (L0 + i) * 16 + 4 * q;
                const uint32_t len = g == kb ? r : 16u;
                const uint32_t off = 16 * g + 4 * q;
                const float4 x = L.stage[par][e * 4 + q];
                const uint32_t bi = pos + (uint32_t)d.idx_offset;
                if (vec && len == 16) {
                    put_pair4(d, off, bi, x);
                } else {
                    const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (uint32_t cc = 0; cc < 4; ++cc) {
                        if (4 * q + cc < len) {
                            put_pair(d, off + cc, bi + cc, xs[cc]);
                        }
                    }
                }
            }
        } else {
            // staging overflowed (low threshold): find the qualifying lines
            // again from src (bit-identical line sums), in order
            uint32_t base = P;
            for (uint32_t i0 = 0; i0 < nl && base < lim; i0 += 64) {
                const uint32_t i = i0 + lane;
                const bool f = i < nl && lane_line_sum(d.src + (size_t)(L0 + i) * 16) >= t;
                const uint64_t m = __ballot(f);
                if (f) {
                    const uint32_t g = base + (uint32_t)__popcll(m & below_mask(lane));
                    if (g < lim) emit_line(d, vec, (L0 + i) * 16, 16 * g, g == kb ? r : 16u);
                }
                base += (uint32_t)__popcll(m);
            }
        }
    }

    // ---- the chunk's window entries at its exchanged offset (used only if
    //      the bucket ends in regime B): line-sum bits, element position, and
    //      the line's index in the reference's candidate vector -- every
    //      non-qualifying line in scan order (thresholdv16.cpp:154,198) ----
    if (Wbef + ww + 1 <= CAND_CAP) {
        const uint32_t nwl = uni(lds_ld(&L.nwl[par]));
        uint32_t *cu = C.cand(b);
        uint32_t *cp = cu + CAND_CAP, *ci = cu + 2 * CAND_CAP;
        const uint32_t tb = f2u(t);
        if (nwl <= WL_B && qw <= STAGE_B) {
            static_assert(WL_B == 64, "one listed entry per lane");
            const uint64_t e = lane < nwl ? L.wl[par][lane] : ~0ull;
            const uint32_t mypos = (uint32_t)e;
            const uint32_t li = mypos / 16 - L0;  // line within the chunk
            uint32_t before = 0, qb = 0;
            for (uint32_t l = 0; l < nwl; ++l) before += (uint32_t)L.wl[par][l] < mypos;
            for (uint32_t x = 0; x < qw; ++x) qb += L.stage_line[par][x] < li;
            if (lane < nwl) {
                const uint32_t idx = Wbef + before;
                st_sc1(&cu[idx], (uint32_t)(e >> 32));
                st_sc1(&cp[idx], mypos);
                st_sc1(&ci[idx], L0 + li - P - qb);
            }
        } else {
            // an LDS list overflowed: list the window from src, in order,
            // counting the qualifying lines before each (as the scan decides:
            // qualifying S >= t, window wlo <= bits(S) < bits(t))
            const uint32_t wlo = tb > WIN ? tb - WIN : 0u;
            uint32_t base = Wbef, qb = P;
            for (uint32_t i0 = 0; i0 < nl; i0 += 64) {
                const uint32_t i = i0 + lane;
                const float S = i < nl ? lane_line_sum(d.src + (size_t)(L0 + i) * 16) : 0.f;
                const uint32_t u = f2u(S);
                const bool qf = i < nl && S >= t;
                const bool wf = i < nl && u >= wlo && u < tb;
                const uint64_t mq = __ballot(qf), mw = __ballot(wf);
                if (wf) {
                    const uint32_t idx = base + (uint32_t)__popcll(mw & below_mask(lane));
                    st_sc1(&cu[idx], u);
                    st_sc1(&cp[idx], (L0 + i) * 16);
                    st_sc1(&ci[idx], L0 + i - (qb + (uint32_t)__popcll(mq & below_mask(lane))));
                }
                base += (uint32_t)__popcll(mw);
                qb += (uint32_t)__popcll(mq);
            }
        }
    }
    release(C, par, j);

    // ---- the bucket's last chunk: regime, tail, AIMD, count, decision ----
    if (c + 1 == d.nc) {
        const uint32_t Qtot = P + qw, Wtot = Wbef + ww;
        const uint32_t c0 = Qtot >= lim ? d.dst_len : 16u * Qtot;
        bool tail_cand = false;
        float tail_key = 0.f;
        uint32_t ct = 0;
        if (c0 < d.dst_len && d.tl) {  // stage 3: the ragged tail's signed, sequential sum
            const float *tp = d.src + (size_t)d.nb * 16;
            float s = 0.f;
            for (uint32_t i = 0; i < d.tl; ++i) s += tp[i];
            s = uni(s);
            if (s * 16.0f >= t * (float)d.tl) ct = std::min(d.dst_len - c0, d.tl);
            else { tail_cand = true; tail_key = s * 16.0f / (float)d.tl; }
        }
        const uint32_t cnt = c0 + ct;
        const bool regimeB = cnt < d.dst_len;
        if (lane == 0) {
            if (ct) {
                const size_t p0 = (size_t)d.nb * 16;
                for (uint32_t i = 0; i < ct; ++i) {
                    put_pair(d, c0 + i, (uint32_t)(p0 + i) + (uint32_t)d.idx_offset, d.src[p0 + i]);
                }
            }
            d.state->t = regimeB ? (float)((double)t * 0.99) : t + inc;
            d.state->inc = inc;
            d.state->init = 1;
            st_sc1(d.count_out, (uint32_t)std::min<uint64_t>(d.dst_len, (uint64_t)d.nb * 16 + d.tl));
            // a bounded wait anywhere in the launch gave up: the output is untrusted
            if (ld_sc1(C.failp)) st_sc1(d.count_out, POISON_COUNT);
        }
        const uint32_t ncand = d.nb - Qtot;  // non-qualifying full lines
        const uint32_t M = regimeB ? std::min((d.dst_len - cnt + 15u) / 16u, ncand) : 0u;
        uint32_t flags = 0;
        if (regimeB) flags = DEC_B | (tail_cand ? DEC_TAIL : 0u) | (Wtot >= M && Wtot + 1 <= CAND_CAP ? DEC_WIN : 0u);
        Decision &D = C.ctl()->dec[b];
        if (lane == 0) {
            st_sc1(&D.w[1], ((uint64_t)cnt << 32) | M);
            st_sc1(&D.w[2], ((uint64_t)Wtot << 32) | __float_as_uint(tail_key));
            st_sc1(&D.w[3], ((uint64_t)Qtot << 32) | __float_as_uint(t));
        }
        vm_drain();
        if (lane == 0) st_sc1(&D.w[0], ((uint64_t)C.tag(TAG_DEC) << 32) | flags);
    }
}

// STAGE (diagnostics only, STG_DEBUG_TV16_STAGE): 0 = full codec; 1 = the
// streaming waves' work only (the finisher releases buffers at once);
// 3 = plain streaming read (calibration).
template <int STAGE, bool EF, bool LONE>
// Registers for 8 waves per SIMD (<= 64 VGPRs): two workgroups per CU take 6
// waves per SIMD and a fill workgroup's 2 run beside them (LONE: 6 waves per
// SIMD, the fill comes after).  The bound says
// 1024 threads (launches use FWG <= 1024) so that the compiler, which derives
// the occupancy it aims for from the bound, does not widen the register
// budget to the 6 waves two FWG-thread workgroups would give.
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(LONE ? 6 : 8, 8)))
tv16_batch(BatchArgs A) {
    __shared__ Lds L;
    Ctx C{A, L, gridDim.x, blockIdx.x, A.ctl, A.cand, A.fail};
    {  // zero the next call's per-call counters (this call never touches them)
        uint32_t *z = reinterpret_cast<uint32_t *>(&A.ctl->cc[(A.epoch + 1) & 1u]);
        constexpr uint32_t words = sizeof(CallCtl) / 4;
        const uint32_t per = (words + C.G - 1) / C.G;
        const uint32_t z0 = C.w * per, z1 = std::min(words, z0 + per);
        for (uint32_t i = z0 + threadIdx.x; i < z1; i += FWG) st_sc1(z + i, 0u);
    }
    if (threadIdx.x < NBUF) {
        L.nst[threadIdx.x] = 0;
        L.nwl[threadIdx.x] = 0;
        L.qcnt[threadIdx.x] = 0;
        L.wcnt[threadIdx.x] = 0;
        L.sdone[threadIdx.x] = 0;
    }
    if (threadIdx.x == 0) {
        L.fdone = 0;
        // slot 0: the next chunk of the call's counter, taken as the
        // workgroup starts; later slots take one each mid-slot.  A
        // workgroup's slots therefore hold increasing chunks, chunks are taken
        // in order, and a chunk is only ever taken by a running workgroup: no
        // wait in this launch points at a workgroup that is not resident.
        L.cid[0] = g_add(&C.cc()->next, 1u);
        for (uint32_t i = 0; i < CIDR; ++i) { L.cok[i] = 0; L.mid[i] = 0; }
        L.cok[0] = 1;
    }
    __syncthreads();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave < NS) {
        for (uint32_t j = 0;; ++j) {
            uint64_t st8 = 0;
            for (uint32_t spins = 0; lds_ld(&L.cok[j % CIDR]) != j + 1; ++spins) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, st8)) { if (flane() == 0) C.spin_fail(6, j, lds_ld(&L.cok[j % CIDR]), wave); break; }
            }
            const uint32_t k = uni(lds_ld(&L.cid[j % CIDR]));
            if (k >= A.K) break;
            asm volatile("" : "+s"(C.w), "+s"(C.G));
            scan_chunk<STAGE, EF, LONE ? SCAN_D_LONE : SCAN_D_BATCH>(C, j, k, wave);
        }
    } else if (wave == FIN) {
        __builtin_amdgcn_s_setprio(3);  // short bursts issue ahead of the streaming waves
        for (uint32_t j = 0;; ++j) {
            uint64_t st9 = 0;
            for (uint32_t spins = 0; lds_ld(&L.cok[j % CIDR]) != j + 1; ++spins) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, st9)) { if (flane() == 0) C.spin_fail(7, j, lds_ld(&L.cok[j % CIDR]), 99); break; }
            }
            const uint32_t k = uni(lds_ld(&L.cid[j % CIDR]));
            if (k >= A.K) break;
            asm volatile("" : "+s"(C.w), "+s"(C.G), "+s"(C.ctlp), "+s"(C.candp), "+s"(C.failp));
            finish_chunk<STAGE>(C, j, k);
        }
    }
}

// Workgroups of a fill launch that order window-miss buckets (tv16wide.h): they
// exit at once when no bucket of the launch needs them.
uint32_t crew_batch() {
    constexpr uint32_t v = 64u;  // > MAX_BATCH: see tv16wide.h crew_loop
    return v;
}
// One-bucket launches: every CU the launch's other workgroups leave (a fill
// workgroup takes a whole CU's LDS), so that phase A streams at full width.
uint32_t crew_lone(uint32_t num_cu, uint32_t others) {
    const uint32_t room = num_cu > others ? num_cu - others : 0u;
    return std::min(std::max(room, MAX_BATCH + 1u), 1024u);
}

}  // namespace

hipError_t launch_tv16(const Tv16Launch &a, const DevWS &ws, hipStream_t s) {
    if (!a.nb) return hipSuccess;
    if (a.nb > MAX_BATCH || !a.epoch || a.epoch >= (1u << 24)) return hipErrorInvalidValue;
    BatchArgs A{};
    Tv16FillArgs F{};
    uint32_t K = 0;
    static const int dbg_stage = getenv("STG_DEBUG_TV16_STAGE") ? atoi(getenv("STG_DEBUG_TV16_STAGE")) : 0;
    constexpr bool lone_ok = true;
    // the one-bucket path: a scan with no waits between workgroups, finished
    // by the fill launch (tv16lone.hip; STG_TV16_LFIN=0: the batched scan)
    static const bool lfin_ok = !(getenv("STG_TV16_LFIN") && atoi(getenv("STG_TV16_LFIN")) == 0);
    auto lone_chunks = [](size_t n) { return std::max<uint32_t>(1, (uint32_t)((n / 16 + LCHUNK - 1) / LCHUNK)); };
    const bool lone_path = lone_ok && lfin_ok && a.nb == 1 && !dbg_stage && lone_chunks(a.b[0].n) <= a.lone_cap &&
                           lone_chunks(a.b[0].n) <= LMAXC && ws.ldesc;
    // a gather-add rides in the one-bucket scan (not on a key's first call,
    // whose threshold is taken from the bucket before the scan); elsewhere it
    // runs as its own pass first
    bool fused_gather = false;
    for (uint32_t i = 0; i < a.nb; ++i) {
        const Tv16Bucket &b = a.b[i];
        if (!b.gather || (!b.gather->resid && b.gather->nsrc <= 1)) continue;  // (no term to add)
        if (b.gather->dst != b.src) return hipErrorInvalidValue;
        if (lone_path && !b.first) {
            fused_gather = true;
        } else {
            const hipError_t e = launch_gather_add(*b.gather, 0, b.n, a.num_cu, s);
            if (e != hipSuccess) return e;
        }
    }
    for (uint32_t i = 0; i < a.nb; ++i) {
        const Tv16Bucket &b = a.b[i];
        if (b.first) {  // first threshold from sequential line sums (thresholdv16.cpp:36-54)
            const uint32_t nblk = (uint32_t)((b.n + 15) / 16);
            tv16_seq_sums<<<(nblk + STG_WG - 1) / STG_WG, STG_WG, 0, s>>>(b.src, b.n, b.sums, nblk);
            const uint32_t bk = std::min<uint32_t>(b.k / 16, nblk - 1);
            hipError_t e = launch_radix_select(b.sums, nblk, 0xffffffffu, 0, bk, ws, a.num_cu, s);
            if (e != hipSuccess) return e;
            tv16_init_state<<<1, 1, 0, s>>>(b.state, ws.rsel);
        }
        BucketDesc &d = A.bk[i];
        d.src = b.src;
        d.idx = b.idx;
        d.val = b.val;
        d.count_out = b.count_out;
        d.state = b.state;
        d.sums_g = b.sums;
        d.resid = b.resid;
        d.nb = (uint32_t)(b.n / 16);
        d.tl = (uint32_t)(b.n % 16);
        d.dst_len = b.dst_len;
        d.idx_offset = b.idx_offset;
        {  // the wire stream is the count = min(dst_len, n) pairs written
            const uint64_t numel = std::min<uint64_t>(b.dst_len, b.n);
            d.wflag = b.wflag & 3u;
            d.wend = numel ? (uint32_t)(8 * ((numel - 1) / 8)) : 0u;
        }
        d.cs = K;
        d.nc = std::max<uint32_t>(1, (d.nb + TV16_CHUNK - 1) / TV16_CHUNK);
        K += d.nc;
        Tv16FillBucket &f = F.bk[i];
        f.src = b.src;
        f.idx = b.idx;
        f.val = b.val;
        f.count_out = b.count_out;
        f.nb = d.nb;
        f.tl = d.tl;
        f.dst_len = d.dst_len;
        f.idx_offset = d.idx_offset;
        f.wflag = d.wflag;
        f.wend = d.wend;
        f.cand = ws.cand + (size_t)i * CAND_WORDS;
        f.heap = reinterpret_cast<uint2 *>(b.sums);
    }
    if (K > a.desc_cap) return hipErrorInvalidValue;
    bool ef = false;  // any bucket with a residual: the fused error-feedback instantiation
    for (uint32_t i = 0; i < a.nb; ++i) ef |= a.b[i].resid != nullptr;
    A.nbk = a.nb;
    A.epoch = a.epoch;
    A.K = K;
    A.ctl = ws.ctl;
    A.desc = ws.desc;
    A.cand = ws.cand;
    A.fail = ws.fail;
    // this launch's share of the device's two scan workgroups per CU
    // (all of them for one stream; launches from several streams split them);
    // no more than there are chunks.  Co-residency is not required.
    const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(std::min<uint32_t>(a.max_wg, K), MAXG));
    const bool lone_scan = lone_ok && a.nb == 1;
    const uint32_t KL = lone_chunks(a.b[0].n);  // one-bucket chunks
    if (lone_path) {
        if (a.ev) (void)hipEventRecord(a.ev[0], s);
        LScanArgs L{};
        L.src = a.b[0].src;
        L.nb = A.bk[0].nb;
        L.nc = KL;
        L.state = a.b[0].state;
        L.cp = ws.cp;
        L.resid = a.b[0].resid;
        L.ldesc = ws.ldesc;
        L.lq = ws.lq;
        L.lw = ws.lw;
        L.lv = ws.lv;
        L.whist = ws.whist;
        L.went = ws.went;
        L.zero_next = reinterpret_cast<uint32_t *>(&ws.ctl->cc[(a.epoch + 1) & 1u]);
        // the window histogram and the finish's arrival block by call parity:
        // this call's copies were zeroed by the previous call's scan
        uint32_t tag = a.epoch;
        if (a.lone_calls) {
            if (++*a.lone_calls == 0) *a.lone_calls = 2;  // (0 is never a tag; the parity keeps alternating)
            tag = *a.lone_calls;
        }
        const uint32_t par = tag & 1u;
        L.whist = ws.whist + (size_t)par * LNBIN;
        L.whist_next = ws.whist + (size_t)(par ^ 1u) * LNBIN;
        L.tag = tag;
        L.done = ws.larr;
        L.tl = (uint32_t)(a.b[0].n % 16);
        // the finish inside the scan launch (tv16lf2.h): not for the wire form
        static const int lf2_env = getenv("STG_TV16_LF2") ? atoi(getenv("STG_TV16_LF2")) : 1;
        // 48 workers + 16 rankers (profiles/r05_lf2_roles_sweep.txt)
        constexpr uint32_t lf2_fin = 64, lf2_wk = 48;
        static_assert(lf2_fin <= LF2_MAXF, "roles");
        {
            static const uint32_t fill_mode0 =
                getenv("STG_DEBUG_TV16_FILL") ? (uint32_t)atoi(getenv("STG_DEBUG_TV16_FILL")) : 0u;
            const bool lf2 = lf2_env != 0 && !a.b[0].wflag && lf2_fin > lf2_wk;
            L.fin = lf2 ? lf2_fin : 0u;
            L.nwk = lf2_wk;
            L.mode = fill_mode0;
            L.out_idx = a.b[0].idx;
            L.out_val = a.b[0].val;
            L.count_out = a.b[0].count_out;
            L.dst_len = a.b[0].dst_len;
            L.idx_offset = a.b[0].idx_offset;
            L.fail = ws.fail;
            L.dbg = ws.misc;
            static const uint32_t skip = getenv("STG_LF2_SKIP") ? (uint32_t)atoi(getenv("STG_LF2_SKIP")) : 0u;
            L.skip = skip;
        }
        if (fused_gather) {  // (fused_gather: bucket 0's gather has a term to add)
            const GatherArgs &g = *a.b[0].gather;
            L.gres = g.resid;
            for (uint32_t x = 1; x < g.nsrc && x < GATHER_MAX; ++x) L.gsrc[x] = g.src[x];
            L.gn = std::max<uint32_t>(1, g.nsrc);
            L.tl = (uint32_t)(a.b[0].n % 16);
        }
        hipError_t e = launch_tv16_lscan(L, a.num_cu, s);  // (clamps L.fin to what the grid allows)
        if (e != hipSuccess) return e;
        if (a.ev) (void)hipEventRecord(a.ev[1], s);
        F.nbk = 1;
        F.epoch = a.epoch;
        F.dec = ws.ctl->dec;
        F.fail = ws.fail;
        F.dbg = ws.misc;
        static const uint32_t fill_mode =
            getenv("STG_DEBUG_TV16_FILL") ? (uint32_t)atoi(getenv("STG_DEBUG_TV16_FILL")) : 0u;
        F.mode = fill_mode;
        F.lone = true;
        constexpr uint32_t workers = 64;
        static const uint32_t rankers = std::max(0, std::min(
            getenv("STG_TV16_LFIN_RANKERS") ? atoi(getenv("STG_TV16_LFIN_RANKERS")) : 8, 128));
        F.helpers = 0;
        F.cc = &ws.ctl->cc[a.epoch & 1u];
        F.lfin = true;
        F.workers = workers;
        F.rankers = rankers;
        F.nc = KL;
        F.ldesc = ws.ldesc;
        F.lq = ws.lq;
        F.lw = ws.lw;
        F.lv = ws.lv;
        F.whist = L.whist;
        F.went = ws.went;
        F.state = a.b[0].state;
        F.cp = ws.cp;
        F.resid = a.b[0].resid;
        F.fin = L.fin;
        F.fin_tag = L.tag;
        F.fin_done = L.done;
        F.crew = crew_lone(a.num_cu, workers + rankers);
        F.crew_ctl = ws.crew;
        if ((e = launch_tv16_fill_any(F, s)) != hipSuccess) return e;
        if (a.ev) (void)hipEventRecord(a.ev[2], s);
        return hipGetLastError();
    }
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    switch (dbg_stage) {
        case 1: tv16_batch<1, false, false><<<G, FWG, 0, s>>>(A); break;
        case 3: tv16_batch<3, false, false><<<G, FWG, 0, s>>>(A); break;
        default:
            if (ef) tv16_batch<0, true, false><<<G, FWG, 0, s>>>(A);
            else if (lone_scan) tv16_batch<0, false, true><<<G, FWG, 0, s>>>(A);
            else tv16_batch<0, false, false><<<G, FWG, 0, s>>>(A);
            break;
    }
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    if (dbg_stage != 1 && dbg_stage != 3) {
        // regime-B heap fill: one workgroup per bucket, stream-ordered after the scan
        F.nbk = a.nb;
        F.epoch = a.epoch;
        F.dec = ws.ctl->dec;
        F.fail = ws.fail;
        F.dbg = ws.misc;
        static const uint32_t fill_mode =
            getenv("STG_DEBUG_TV16_FILL") ? (uint32_t)atoi(getenv("STG_DEBUG_TV16_FILL")) : 0u;
        F.mode = fill_mode;
        F.lone = lone_scan;
        F.helpers = F.lone ? 15u : 0u;
        F.cc = &ws.ctl->cc[a.epoch & 1u];
        F.crew = F.lone ? crew_lone(a.num_cu, F.nbk + F.helpers) : crew_batch();
        F.crew_ctl = ws.crew;
        const hipError_t e = launch_tv16_fill_any(F, s);
        if (e != hipSuccess) return e;
    }
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}

}  // namespace stg
