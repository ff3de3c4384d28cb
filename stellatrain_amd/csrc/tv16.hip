// tv16.hip -- thresholdv16 ("cache-aware" threshold-v) on gfx950.
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
// lines in descending-sum order (heap fill).  AIMD: t *= 0.99 (in double) when
// the scan ran dry, t += inc otherwise.
//
// One persistent launch per batch of buckets (tv16_batch).  The buckets are
// cut into 2048-line chunks (128 KiB), taken in order by 1024-thread
// workgroups (2 per CU, all co-resident) from a per-call counter, so fast
// workgroups take more chunks and every dependency below points backward in
// time.  The 16 waves of a workgroup are specialised:
//
//   14 streaming waves  scan chunk after chunk and never wait on another
//             workgroup: stream the chunk once (a quad of lanes per line, DPP
//             cross-lane adds in the AVX tree order), stage the qualifying
//             lines' data in LDS with one ballot per 16-line step (their
//             in-chunk order), list the lines in a window just below t, and
//             count both; the last wave done with a chunk publishes its
//             aggregate counts.  They stall only when NBUF chunks ahead of
//             the finisher (LDS buffer sets in use).
//   finisher wave  per chunk: decoupled look-back over the bucket's earlier
//             chunks for the prefix counts, publish the inclusive prefix,
//             emit the chunk's qualifying lines with rank < kb (+1 partial)
//             straight from LDS, write its window list at its window offset;
//             the bucket's last chunk decides the regime and writes the tail,
//             the AIMD threshold, the count and the decision.
//   ranker wave    per bucket decided regime B: wait for every chunk's window
//             list, rank this workgroup's share of the set and emit it in
//             (sum desc, position asc) order.  When the window does not hold
//             the top M it runs a radix descent over the bucket's line sums
//             with grid barriers among the rankers.
//
// A key's first call runs tv16_seq_sums + a radix select (select.hip) before
// the launch.
#include <algorithm>
#include <cstdlib>

#include "ws.h"

namespace stg {

namespace {

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
#ifndef STG_EF_AUX
#define STG_EF_AUX 2  // cache policy of the fused residual stores (2: nontemporal)
#endif

constexpr uint32_t FWG = 1024;      // workgroup: 16 waves
constexpr uint32_t FNW = FWG / 64;
constexpr uint32_t NS = FNW - 2;    // streaming waves 0..13
constexpr uint32_t FIN = NS;        // wave 14: finisher
constexpr uint32_t RNK = NS + 1;    // wave 15: ranker (regime-B heap fill)
static_assert(RNK == FNW - 1, "one streaming group, one finisher, one ranker");
#ifndef STG_TV16_NBUF
#define STG_TV16_NBUF 5
#endif
#ifndef STG_TV16_SCAN_D
#define STG_TV16_SCAN_D 3
#endif
constexpr uint32_t NBUF = STG_TV16_NBUF;  // LDS buffer sets (slots) in flight per workgroup
constexpr uint32_t CIDR = 2 * NBUF;       // chunk-id ring
#ifndef STG_TV16_STAGE_B
#define STG_TV16_STAGE_B 72
#endif
#ifndef STG_TV16_WL_B
#define STG_TV16_WL_B 64
#endif
constexpr uint32_t STAGE_B = STG_TV16_STAGE_B;  // qualifying lines staged in LDS per slot (~20 expected at 1%)
constexpr uint32_t WL_B = STG_TV16_WL_B;  // window candidates listed in LDS per slot
#ifndef STG_TV16_POLL_SLEEP
#define STG_TV16_POLL_SLEEP 8  // s_sleep units (64 clocks) between prefix polls
#endif
// diagnostics only (timing attribution; wrong results): skip the prefix waits
// or the ordered emission
#ifndef STG_TV16_DIAG_NOWAIT
#define STG_TV16_DIAG_NOWAIT 0
#endif
#ifndef STG_TV16_DIAG_NOEMIT
#define STG_TV16_DIAG_NOEMIT 0
#endif
#ifndef STG_TV16_DIAG_STORES
#define STG_TV16_DIAG_STORES 0
#endif
#ifndef STG_TV16_LAST_FLUSH
#define STG_TV16_LAST_FLUSH 1
#endif
#ifndef STG_TV16_DEC_SLEEP
#define STG_TV16_DEC_SLEEP 16  // between a ranker's polls of the next decision
#endif
#ifndef STG_TV16_PRIO
#define STG_TV16_PRIO 1
#endif
#ifndef STG_TV16_RK
#define STG_TV16_RK 64
#endif
constexpr uint32_t RK = STG_TV16_RK; // rankers per regime-B bucket (window path)
constexpr uint32_t WBINS = 1024;    // window-path counting sort: bins over the top 10 key bits
constexpr uint32_t GB = 512;        // chunk descriptors gathered per round trip (a 64 MiB bucket has 512)
// float4 loads in flight per streaming wave: 2 x 14 x 64 x 16 B x SCAN_D per CU
// (SCAN_D = 3: 84 KiB per CU, just over the ~72 KiB that hides an HBM miss;
// deeper queues add latency to every exchange round trip -- Little's law)
constexpr uint32_t SCAN_D = STG_TV16_SCAN_D;
constexpr uint32_t MAXG = 512;      // workgroups per launch (2 per CU)
constexpr uint32_t L1_SHIFT = 14;   // level-1 bin width in ulps below t (~0.2% of t)
constexpr uint32_t WIN = 1u << 17;  // regime-B window below t, in ulps (~1.6% of t)
// Bounded waits give up after SPIN_TICKS of the 100 MHz s_memrealtime clock
// (read every 64 polls, from the first poll on): the same wall-clock limit at
// every site, so the wait that started first also gives up first.
constexpr uint64_t SPIN_TICKS = 20000000;  // 200 ms
__device__ __forceinline__ bool spin_expired(uint32_t spins, uint64_t &t0) {
    if (spins & 63u) return false;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (spins == 0) { t0 = now; return false; }
    return now - t0 > SPIN_TICKS;
}
static_assert(SORT_CAP == MAX_BATCH * CAND_CAP, "one candidate slot per bucket of a launch");

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
struct BucketDesc {  // 80 bytes
    const float *src;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    float *sums_g;  // line sums, materialised by the rankers' rare paths
    uint32_t nb, tl, dst_len;
    int32_t idx_offset;
    uint32_t cs, nc;  // chunks [cs, cs + nc) of the launch's chunk sequence (nc >= 1)
    float *resid;     // fused error feedback: the streaming waves copy every full line here (or null)
};

struct BatchArgs {
    BucketDesc bk[MAX_BATCH];
    uint32_t nbk;
    uint32_t epoch;  // 1 .. 2^24-1
    uint32_t K;      // chunks in the launch
    FillCtl *ctl;
    ChunkDesc *desc;
    uint64_t *cand;
    uint32_t *fail;
    uint32_t *stamps;  // STAGE 4 diagnostics: 128 words per workgroup
};

// LDS of one workgroup (< 80 KiB: two workgroups per CU).
struct Lds {
    // streaming waves -> finisher, by buffer set (slot % NBUF)
    float4 stage[NBUF][STAGE_B * 4];     // staged qualifying lines (64 B each)
    uint32_t stage_line[NBUF][STAGE_B];
    uint64_t wl[NBUF][WL_B];             // window candidates, composite keys
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
    uint32_t pw[MAX_BATCH];              // window lines of the pending (uncounted) lists, by bucket
    uint32_t cum[MAX_BATCH];             // counted so far, by bucket: chunks << 16 | window lines
    // ranker
    union {
        uint64_t cand[CAND_CAP];         // rare path: candidate set (u64 composite keys)
        uint32_t hist[HBINS];            // rare path: radix descent
        struct {                         // window path: counting-sort rank of 32-bit keys
            uint32_t key[CAND_CAP];      // the set, as gathered
            uint32_t srt[CAND_CAP];      // the set sorted by top bits (bin order)
            uint32_t bin[WBINS];         // bin counts -> bin ends
            uint4 ent[64];               // this ranker's entries: {rank, pos, len, off}
        } wr;
    };
    uint32_t stamp[128];                 // STAGE 4 diagnostics only
};

__device__ __forceinline__ uint32_t bitlen(uint32_t x) { return x ? 32u - __clz(x) : 0u; }

// Wave-uniform values read from memory or LDS: move them to SGPRs.
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ float uni(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

// lane id, opaque to the compiler (not hoisted into a live register)
__device__ __forceinline__ uint32_t flane() {
    uint32_t x;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
    return x;
}
__device__ __forceinline__ uint64_t below_mask(uint32_t lane) { return lane ? (~0ull >> (64 - lane)) : 0ull; }

// LDS hand-offs between the waves of one workgroup: the writer drains its
// LDS operations before the flag; LDS executes one wave's operations in order.
__device__ __forceinline__ void lds_drain() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t lds_ld(const uint32_t *p) {
    return __hip_atomic_load(const_cast<uint32_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Tree sum of one 16-float line held as a float4 by each lane of a quad
// (lanes 0,1: floats 0..7; lanes 2,3: floats 8..15): p = |x_i| + |x_{i+4}|,
// h = (p0+p1)+(p2+p3) per half, S = h_lo + h_hi  (thresholdv16.cpp:57-73,143).
__device__ __forceinline__ float quad_line_sum(const float4 v) {
    const float ax = fabsf(v.x), ay = fabsf(v.y), az = fabsf(v.z), aw = fabsf(v.w);
    const float px = ax + dpp_f<QP_XOR1>(ax);
    const float py = ay + dpp_f<QP_XOR1>(ay);
    const float pz = az + dpp_f<QP_XOR1>(az);
    const float pw = aw + dpp_f<QP_XOR1>(aw);
    const float h = (px + py) + (pz + pw);
    return h + dpp_f<QP_XOR2>(h);
}

// The same sum by one lane from memory (bit-identical: the same adds in the
// same order; IEEE addition is commutative).
__device__ __forceinline__ float lane_line_sum(const float *p) {
    const float4 *p4 = reinterpret_cast<const float4 *>(p);
    const float4 a = p4[0], b = p4[1], c = p4[2], e = p4[3];
    const float lo = ((fabsf(a.x) + fabsf(b.x)) + (fabsf(a.y) + fabsf(b.y))) +
                     ((fabsf(a.z) + fabsf(b.z)) + (fabsf(a.w) + fabsf(b.w)));
    const float hi = ((fabsf(c.x) + fabsf(e.x)) + (fabsf(c.y) + fabsf(e.y))) +
                     ((fabsf(c.z) + fabsf(e.z)) + (fabsf(c.w) + fabsf(e.w)));
    return lo + hi;
}

// Composite heap-fill key: ascending order = (sum desc, position asc).
__device__ __forceinline__ uint64_t cand_key(uint32_t u, uint32_t pos) {
    return ((uint64_t)(~(u | 0x80000000u)) << 32) | (uint64_t)pos;
}

// One lane writes `len` (<= 16) pairs of the line at `pos` to slot `off`.
__device__ __forceinline__ void emit_line(const BucketDesc &d, bool vec, uint32_t pos, uint32_t off, uint32_t len) {
    if (vec && len == 16) {
        const float4 *s4 = reinterpret_cast<const float4 *>(d.src + pos);
        float4 *v4 = reinterpret_cast<float4 *>(d.val + off);
        uint4 *i4 = reinterpret_cast<uint4 *>(d.idx + off);
        const uint32_t b = pos + (uint32_t)d.idx_offset;
        const float4 x0 = s4[0], x1 = s4[1], x2 = s4[2], x3 = s4[3];
        v4[0] = x0; v4[1] = x1; v4[2] = x2; v4[3] = x3;
        i4[0] = make_uint4(b + 0, b + 1, b + 2, b + 3);
        i4[1] = make_uint4(b + 4, b + 5, b + 6, b + 7);
        i4[2] = make_uint4(b + 8, b + 9, b + 10, b + 11);
        i4[3] = make_uint4(b + 12, b + 13, b + 14, b + 15);
    } else {
        for (uint32_t i = 0; i < len; ++i) {
            d.val[off + i] = d.src[(size_t)pos + i];
            d.idx[off + i] = pos + i + (uint32_t)d.idx_offset;
        }
    }
}

__device__ __forceinline__ bool aligned16(const BucketDesc &d) {
    return ((reinterpret_cast<uintptr_t>(d.src) | reinterpret_cast<uintptr_t>(d.idx) |
             reinterpret_cast<uintptr_t>(d.val)) & 15u) == 0;
}

// `n16` 16-byte words from global memory (read through to L2: sc1) into LDS
// at `dst`, in chunks of 64 (the destination must hold whole chunks); waits.
__device__ __forceinline__ void gather16(const void *src, uint32_t n16, void *dst) {
    const uint32_t lane = flane();
    for (uint32_t c = 0; c * 64 < n16; ++c) {
        const uint32_t v = std::min(c * 64 + lane, n16 - 1);
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const char *>(src) + (size_t)v * 16,
                                         reinterpret_cast<char *>(dst) + c * 1024, 16, 0, 16 /* sc1 */);
    }
    vm_drain();
}

// Spin-timeout failure bits: FAIL_SPIN_TIMEOUT plus bit 8 + site naming the
// wait that gave up: 0 grid barrier, 1 buffer set, 2 prefix aggregates,
// 3 chunk streamed, 4 decision, 5 window lists, 6 / 7 slot chunk id
// (streamer / finisher), 8 the previous slot's chunk take.
__device__ __forceinline__ constexpr uint32_t spin_site(uint32_t site) { return FAIL_SPIN_TIMEOUT | (1u << (8 + site)); }

struct Ctx {
    const BatchArgs &A;
    Lds &L;
    uint32_t G, w;
    uint32_t nbar;  // ranker: grid-barrier rounds used so far (the same in every ranker)
    FillCtl *ctlp;
    uint64_t *candp;
    uint32_t *failp;
    bool stamping;  // STAGE 4

    __device__ __forceinline__ uint32_t tag(uint32_t kind) const { return (A.epoch << 8) | kind; }
    __device__ __forceinline__ FillCtl *ctl() const { return ctlp; }
    __device__ __forceinline__ CallCtl *cc() const { return &ctlp->cc[A.epoch & 1u]; }
    __device__ __forceinline__ uint64_t *cand(uint32_t b) const { return candp + (size_t)b * CAND_CAP; }
    __device__ __forceinline__ void fail(uint32_t bits) const { g_or(failp, bits); }
    // A spin timeout: its site bit, and for the first one in the workspace's
    // life a record for the host's error message: {site + 1, workgroup, x0,
    // x1, x2, epoch} at fail[1..6]; per site, its first one at fail[8 + 4 site].
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
    }
    __device__ __forceinline__ void stamp(uint32_t slot, uint32_t v) const {
        if (stamping && slot < 128 && flane() == 0) L.stamp[slot] = v ? v : (uint32_t)__builtin_amdgcn_s_memrealtime();
    }
    // bucket holding global chunk k (scalar search over <= 16 buckets)
    __device__ __forceinline__ uint32_t bucket_of(uint32_t k) const {
        uint32_t b = 0;
        while (b + 1 < A.nbk && k >= A.bk[b + 1].cs) ++b;
        return b;
    }

    // Grid barrier among the ranker waves (one per workgroup): the wave whose
    // arrival completes round r writes every workgroup's own go word; each
    // ranker polls only its own.  Bounded.
    __device__ __forceinline__ void grid_sync() {
        const uint32_t r = ++nbar;
        FillCtl *fc = ctl();
        const uint64_t go = ((uint64_t)(A.epoch << 8) << 32) | r;
        const uint32_t lane = flane();
        vm_drain();
        uint32_t old = 0;
        if (lane == 0) old = g_add(&cc()->bar, 1u);
        old = uni(old);
        if (old == r * G - 1) {
            for (uint32_t i = lane; i < G; i += 64) st_sc1(&fc->slot[i].go, go);
            vm_drain();
        }
        uint64_t st1 = 0;
        for (uint32_t spins = 0; ld_sc1(&fc->slot[w].go) != go; ++spins) {
            __builtin_amdgcn_s_sleep(1);
            if (spin_expired(spins, st1)) { if (lane == 0) spin_fail(0, r, ld_acq_relaxed(&cc()->bar), G); break; }
        }
    }
};

constexpr uint32_t TAG_AGG = 1, TAG_DEC = 3, TAG_TIE = 4, TAG_RDY = 5, TAG_LST = 6;
constexpr uint32_t DEC_B = 1, DEC_WIN = 2, DEC_TAIL = 4;

// ===========================================================================
// streaming waves
// ===========================================================================
// scan of slot j = chunk k by streaming wave s: lines i = (s + NS*m)*16 +
// lane/4 of the chunk, m = 0, 1, ...; SCAN_D float4 loads per lane in flight
// through a buffer descriptor bounded to the chunk (lanes past it read zeros).
template <int STAGE, bool EF>
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
        if (C.stamping && spins && flane() == 0) atomicAdd(&L.stamp[120], spins);
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
        __builtin_amdgcn_raw_buffer_store_b128(t4, rsrc_r, voff + m * (NS * 1024u), 0, STG_EF_AUX /* 2 = nt */);
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
    // The first wave past the middle of slot j takes the chunk of slot j + 2
    // from the call's counter (slots 0 and 1 are static): late enough that
    // chunks are taken close to when they are streamed (the finishers' prefix
    // counts wait on earlier chunks only), early enough that the round trip
    // hides behind the second half of the slot.  A take waits until slot
    // j - 1's take is published (slot j + 1's chunk id), so a workgroup's
    // chunk ids increase slot by slot and the first id >= K ends it with no
    // chunk left behind -- a wave with no steps in a short chunk could
    // otherwise run ahead into slot j + 1 and take before slot j did.
    uint32_t nx = 0;
    bool grab = false, tried = false;
    auto try_take = [&]() {
        tried = true;
        uint32_t first = 1;
        if (flane() == 0) first = atomicAdd(&L.mid[j % CIDR], 1u);
        grab = uni(first) == 0;
        if (grab && flane() == 0) nx = 2 * C.G + g_add(&C.cc()->next, 1u);
    };
    auto prev_taken = [&]() { return lds_ld(&L.cok[(j + 1) % CIDR]) == j + 2; };
    for (uint32_t m0 = 0; m0 < mine; m0 += SCAN_D) {
        if (!tried && m0 >= mine / 2 && prev_taken()) try_take();
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
                    if (slot < WL_B) L.wl[par][slot] = cand_key(us, (L0 + i) * 16);
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
    if (!tried) {  // no steps here (a short chunk) or slot j - 1's take came late
        uint64_t st3 = 0;
        for (uint32_t spins = 0; !prev_taken(); ++spins) {
            __builtin_amdgcn_s_sleep(1);
            if (spin_expired(spins, st3)) { if (flane() == 0) C.spin_fail(8, j, lds_ld(&L.cok[(j + 1) % CIDR]), s); break; }
        }
        try_take();
    }
    if (grab && flane() == 0) {
        // slot j + NBUF reuses slot j - NBUF's counter: every wave is done
        // with slot j - NBUF (the finisher released it) and none is past j yet
        L.mid[(j + NBUF) % CIDR] = 0;
        L.cid[(j + 2) % CIDR] = nx;
        lds_drain();
        lds_st(&L.cok[(j + 2) % CIDR], j + 3);
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
                if (!pm || STG_TV16_DIAG_NOWAIT) break;
                const uint32_t hl = 63u - (uint32_t)__clzll((long long)pm);
                __builtin_amdgcn_s_sleep(STG_TV16_POLL_SLEEP);
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

// Per-finisher state carried between slots: window lists written but not yet
// counted (their stores are retired by the next gather), 4 bits per bucket;
// their window lines are summed in L.pw.
struct FinState {
    uint64_t pend;
};

// Count the pending window lists as in place (the caller drained its stores).
__device__ __forceinline__ void flush_lists(Ctx &C, FinState &F) {
    for (uint32_t b = 0; F.pend; ++b, F.pend >>= 4) {
        const uint32_t n = (uint32_t)(F.pend & 15u);
        if (n && flane() == 0) {
            // this workgroup's own line: no other workgroup writes it
            const uint32_t c0 = C.L.cum[b];
            const uint32_t ch = (c0 >> 16) + n, wl = std::min(0xffffu, (c0 & 0xffffu) + C.L.pw[b]);
            C.L.cum[b] = (ch << 16) | wl;
            C.L.pw[b] = 0;
            st_sc1(&C.ctl()->lst[C.w].w[b], ((uint64_t)C.tag(TAG_LST) << 32) | (ch << 16) | wl);
        }
    }
}

// finish(slot j = chunk k): look-back, ordered emission, window list; the
// bucket's last chunk also decides the regime, writes tail / AIMD / count and
// posts the decision for the rankers.
template <int STAGE>
__device__ __forceinline__ void finish_chunk(Ctx &C, uint32_t j, uint32_t k, FinState &F) {
    Lds &L = C.L;
    const uint32_t par = j % NBUF;
    const uint32_t lane = flane();
    if (F.pend && lds_ld(&L.sdone[par]) < NS) {
        // idle until the chunk is streamed: retire and count the pending
        // window lists now (the rankers wait for them)
        vm_drain();
        flush_lists(C, F);
    }
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
    if (j < 16) C.stamp(j * 4 + 0, 0);

    // ---- prefix counts of the bucket's earlier chunks ----
    uint32_t P = 0, Wbef = 0;
    if (c) {
        prefix_counts(C, b, c, P, Wbef);
        flush_lists(C, F);  // the gather retired the earlier chunks' list stores
    }
    const uint32_t ww = uni(L.wcnt[par]);
    if (j < 16) C.stamp(j * 4 + 1, 0);

    // ---- ordered emission of the chunk's qualifying lines with rank < lim ----
    const uint32_t kb = d.dst_len / 16, r = d.dst_len % 16;
    const uint32_t lim = kb + (r ? 1u : 0u);
    const bool vec = aligned16(d);
    if (P < lim && qw && !STG_TV16_DIAG_NOEMIT) {
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
                    *reinterpret_cast<float4 *>(d.val + off) = x;
                    *reinterpret_cast<uint4 *>(d.idx + off) = make_uint4(bi, bi + 1, bi + 2, bi + 3);
                } else {
                    const float xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (uint32_t cc = 0; cc < 4; ++cc) {
                        if (4 * q + cc < len) {
                            d.val[off + cc] = xs[cc];
                            d.idx[off + cc] = bi + cc;
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

    // ---- the chunk's window candidates at its exchanged offset (speculative:
    //      used only if the bucket ends in regime B with the window path) ----
    if (STAGE != 5 && Wbef + ww + 1 <= CAND_CAP) {
        // 32-bit window keys (tb-1-u) << 12 | set index, the set in position
        // order (chunks in order, each list sorted by position), plus the
        // line positions at [CAND_CAP + index]
        const uint32_t nwl = uni(lds_ld(&L.nwl[par]));
        uint32_t *ckey = reinterpret_cast<uint32_t *>(C.cand(b));
        uint32_t *cpos = ckey + CAND_CAP;
        const uint32_t tb = f2u(t);
        if (nwl <= WL_B) {
            const uint64_t e = lane < nwl ? L.wl[par][lane] : ~0ull;
            const uint32_t mypos = (uint32_t)e;
            uint32_t before = 0;
            for (uint32_t l = 0; l < nwl; ++l) before += (uint32_t)L.wl[par][l] < mypos;
            if (lane < nwl) {
                const uint32_t u = ~(uint32_t)(e >> 32) & 0x7fffffffu;
                const uint32_t idx = Wbef + before;
                st_sc1(&ckey[idx], ((tb - 1u - u) << 12) | idx);
                st_sc1(&cpos[idx], mypos);
            }
        } else {  // the LDS list overflowed: list the window from src, in order
            const uint32_t wlo = tb > WIN ? tb - WIN : 0u;
            uint32_t base = Wbef;
            for (uint32_t i0 = 0; i0 < nl; i0 += 64) {
                const uint32_t i = i0 + lane;
                const uint32_t u = i < nl ? f2u(lane_line_sum(d.src + (size_t)(L0 + i) * 16)) : 0xffffffffu;
                const bool p = u >= wlo && u < tb;
                const uint64_t m = __ballot(p);
                if (p) {
                    const uint32_t idx = base + (uint32_t)__popcll(m & below_mask(lane));
                    st_sc1(&ckey[idx], ((tb - 1u - u) << 12) | idx);
                    st_sc1(&cpos[idx], (L0 + i) * 16);
                }
                base += (uint32_t)__popcll(m);
            }
        }
    }
    if (j < 16) C.stamp(j * 4 + 3, 0);
#pragma unroll
    for (uint32_t x = 0; x < STG_TV16_DIAG_STORES; ++x) st_sc1(C.failp + 60 + (x & 3), 0u);  // diagnostics: extra stores
    if (((F.pend >> (4 * b)) & 15u) == 15u) {  // counter full: retire and count now
        vm_drain();
        flush_lists(C, F);
    }
    F.pend += 1ull << (4 * b);
    if (lane == 0) L.pw[b] += ww;
    if (STG_TV16_LAST_FLUSH && c + 1 == d.nc) {  // the bucket's last list: count it now, the rankers wait for it
        vm_drain();
        flush_lists(C, F);
    }
    release(C, par, j);
    if (j < 16) C.stamp(j * 4 + 2, 0);

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
                    d.val[c0 + i] = d.src[p0 + i];
                    d.idx[c0 + i] = (uint32_t)(p0 + i) + (uint32_t)d.idx_offset;
                }
            }
            d.state->t = regimeB ? (float)((double)t * 0.99) : t + inc;
            d.state->inc = inc;
            d.state->init = 1;
            *d.count_out = (uint32_t)std::min<uint64_t>(d.dst_len, (uint64_t)d.nb * 16 + d.tl);
        }
        const uint32_t ncand = d.nb - Qtot;  // non-qualifying full lines
        const uint32_t M = regimeB ? std::min((d.dst_len - cnt + 15u) / 16u, ncand) : 0u;
        uint32_t flags = 0;
        if (regimeB && STAGE != 5) {
            flags = DEC_B | (tail_cand ? DEC_TAIL : 0u) | (M > 0 && Wtot >= M && Wtot + 1 <= CAND_CAP ? DEC_WIN : 0u);
        }
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

// ===========================================================================
// ranker wave: the regime-B heap fill, top candidates by (sum desc, pos asc)
// ===========================================================================
// Rank-and-emit of a collected candidate set: output order is ascending
// composite key; an entry's rank is the number of smaller keys.  Ranker r of
// the R taking part ranks entries r, r + R, ... (8 at a time) in one pass over
// an LDS copy of the set (+ the ragged tail when it competes).
__device__ __forceinline__ void rank_emit(Ctx &C, uint32_t r, uint32_t R, const BucketDesc &d, const uint64_t *cand,
                                          uint32_t cnt, uint32_t nc_all, bool add_tail, float tail_key) {
    Lds &L = C.L;
    const uint32_t total = nc_all + (add_tail ? 1u : 0u);
    if (r >= total) return;
    const uint32_t lane = flane();
    const uint32_t tailpos = d.nb * 16;
    const uint64_t tail_comp = ((uint64_t)(~ford(tail_key)) << 32) | (uint64_t)tailpos;
    if (nc_all) gather16(cand, (nc_all + 1) / 2, L.cand);
    if (add_tail && lane == 0) L.cand[nc_all] = tail_comp;
    lds_drain();
    constexpr uint32_t KB = 8;
    const uint32_t ne = (total - r + R - 1) / R;
    for (uint32_t k0 = 0; k0 < ne; k0 += KB) {
        uint64_t key[KB];
        uint32_t less[KB];
#pragma unroll
        for (uint32_t k = 0; k < KB; ++k) {
            const uint32_t e = r + (k0 + k) * R;
            key[k] = k0 + k < ne ? L.cand[e] : 0ull;
            key[k] = ((uint64_t)uni((uint32_t)(key[k] >> 32)) << 32) | uni((uint32_t)key[k]);
            less[k] = 0;
        }
        for (uint32_t jj = lane; jj < total; jj += 64) {
            const uint64_t x = L.cand[jj];
#pragma unroll
            for (uint32_t k = 0; k < KB; ++k) less[k] += x < key[k];
        }
#pragma unroll
        for (uint32_t k = 0; k < KB; ++k) {
            if (k0 + k >= ne) break;
            const uint32_t rank = wave_sum(less[k]);
            const bool is_tail = add_tail && key[k] == tail_comp;
            const bool tail_before = add_tail && tail_comp < key[k];
            const uint32_t pos = (uint32_t)key[k];
            const uint32_t len = is_tail ? d.tl : 16u;
            const uint64_t off = (uint64_t)cnt + 16ull * rank - (tail_before ? (uint64_t)(16u - d.tl) : 0ull);
            if (off < d.dst_len) {
                const uint32_t Ln = std::min<uint32_t>(len, d.dst_len - (uint32_t)off);
                if (lane < Ln) {
                    d.val[off + lane] = d.src[(size_t)pos + lane];
                    d.idx[off + lane] = pos + lane + (uint32_t)d.idx_offset;
                }
            }
        }
    }
}

// Window path rank-and-emit.  The set holds Wtot unique 32-bit keys
// (tb-1-u) << 12 | index, ascending = (sum desc, position asc), index in
// position order.  Each ranker gathers it into LDS, counting-sorts it by the
// top 10 bits (LDS atomics), and ranks its entries r, r + R, ... as bin start
// + the smaller keys of the same bin (a few); the ragged tail competes as
// index Wtot when its key falls inside the window.
__device__ __forceinline__ void rank_window(Ctx &C, uint32_t r, uint32_t R, const BucketDesc &d, uint32_t b,
                                            uint32_t cnt, uint32_t Wtot, bool tail, float tail_key, uint32_t tb) {
    Lds &L = C.L;
    const uint32_t lane = flane();
    const uint32_t *ckey = reinterpret_cast<const uint32_t *>(C.cand(b));
    const uint32_t *cpos = ckey + CAND_CAP;
    const uint32_t wlo = tb > WIN ? tb - WIN : 0u;
    const uint32_t ut = f2u(tail_key);  // a negative tail key has the sign bit: never in the window
    const bool tail_in = tail && ut >= wlo && ut < tb && Wtot < CAND_CAP;
    const uint32_t tail_k = ((tb - 1u - ut) << 12) | Wtot;
    if (Wtot) gather16(ckey, (Wtot + 3) / 4, L.wr.key);
    const uint32_t total = Wtot + (tail_in ? 1u : 0u);
    if (tail_in && lane == 0) L.wr.key[Wtot] = tail_k;
    for (uint32_t i = lane; i < WBINS; i += 64) L.wr.bin[i] = 0;
    lds_drain();
    constexpr uint32_t SH = 29 - 10;  // keys < 2^29
    for (uint32_t i = lane; i < total; i += 64) atomicAdd(&L.wr.bin[L.wr.key[i] >> SH], 1u);
    lds_drain();
    {  // exclusive scan of the bins, 16 per lane (read twice: no register array)
        constexpr uint32_t BPL = WBINS / 64;
        uint32_t sum = 0;
        for (uint32_t q = 0; q < BPL; ++q) sum += L.wr.bin[lane * BPL + q];
        uint32_t run = wave_incl_scan(sum) - sum;
        for (uint32_t q = 0; q < BPL; ++q) {
            const uint32_t c = L.wr.bin[lane * BPL + q];
            L.wr.bin[lane * BPL + q] = run;
            run += c;
        }
    }
    lds_drain();
    for (uint32_t i = lane; i < total; i += 64) {
        const uint32_t k = L.wr.key[i];
        L.wr.srt[atomicAdd(&L.wr.bin[k >> SH], 1u)] = k;  // bin[x] ends as the end of bin x
    }
    lds_drain();
    const uint32_t ne = (total - r + R - 1) / R;
    const bool vec = aligned16(d);
    const uint32_t tailpos = d.nb * 16;
    for (uint32_t e0 = 0; e0 < ne; e0 += 64) {
        // one entry per lane: its rank, position, length and output offset
        const uint32_t q = e0 + lane;
        if (q < ne) {
            const uint32_t k = L.wr.key[r + q * R];
            const uint32_t bn = k >> SH;
            const uint32_t lo = bn ? L.wr.bin[bn - 1] : 0u, hi = L.wr.bin[bn];
            uint32_t rank = lo;
            for (uint32_t x = lo; x < hi; ++x) rank += L.wr.srt[x] < k;
            const uint32_t idx = k & 0xfffu;
            const bool is_tail = tail_in && idx == Wtot;
            const bool tail_before = tail_in && tail_k < k;
            const uint64_t off = (uint64_t)cnt + 16ull * rank - (tail_before ? (uint64_t)(16u - d.tl) : 0ull);
            const uint32_t pos = is_tail ? tailpos : ld_sc1(&cpos[idx]);
            const uint32_t len = off < d.dst_len ? std::min<uint32_t>(is_tail ? d.tl : 16u, d.dst_len - (uint32_t)off) : 0u;
            L.wr.ent[lane] = make_uint4(rank, pos, len, (uint32_t)std::min<uint64_t>(off, 0xffffffffu));
        }
        lds_drain();
        // emission: a quad of lanes per entry, two groups of 16 entries in
        // flight (their loads issued before their stores)
        const uint32_t nq = std::min(64u, ne - e0);
        const uint32_t c4 = 4 * (lane & 3);
        for (uint32_t g0 = 0; g0 < 4; g0 += 2) {
            float4 x[2];
            uint4 en[2];
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t el = (g0 + h) * 16 + (lane >> 2);
                en[h] = el < nq ? L.wr.ent[el] : make_uint4(0, 0, 0, 0);
                x[h] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (en[h].z == 16 && vec) x[h] = *reinterpret_cast<const float4 *>(d.src + (size_t)en[h].y + c4);
            }
#pragma unroll
            for (uint32_t h = 0; h < 2; ++h) {
                const uint32_t len = en[h].z, pos = en[h].y, off = en[h].w;
                if (!len) continue;
                const uint32_t bi = pos + c4 + (uint32_t)d.idx_offset;
                if (len == 16 && vec) {
                    *reinterpret_cast<float4 *>(d.val + off + c4) = x[h];
                    *reinterpret_cast<uint4 *>(d.idx + off + c4) = make_uint4(bi, bi + 1, bi + 2, bi + 3);
                } else {
                    for (uint32_t cc = 0; cc < 4; ++cc) {
                        if (c4 + cc < len) {
                            d.val[off + c4 + cc] = d.src[(size_t)pos + c4 + cc];
                            d.idx[off + c4 + cc] = bi + cc;
                        }
                    }
                }
            }
        }
        lds_drain();
    }
}

// Rare paths: the window does not hold the top M -> radix descent over the
// bucket's line sums (ranker w takes chunks w, w + G, ...; sums recomputed
// from src into sums_g) with grid barriers among the rankers, then rank and
// emit.  The top M lines are taken in pieces of at most CAND_CAP - 1
// candidates (the LDS rank capacity), in output order: each piece is the
// next run of keys below the previous piece's cut, so a large M (the count
// fell far short of k) is emitted piece by piece at increasing offsets.
__device__ __forceinline__ void rank_rare(Ctx &C, uint32_t b, uint32_t flags, uint32_t cnt, uint32_t M, float t,
                                          float tail_key) {
    const BucketDesc &d = C.A.bk[b];
    Lds &L = C.L;
    const uint32_t G = C.G, w = C.w, lane = flane();
    const bool vec = aligned16(d);
    const uint32_t tb = f2u(t);
    uint64_t *cand = C.cand(b);
    BucketCtl *bc = &C.cc()->bk[b];
    // this ranker's lines: chunks c = w, w + G, ... of the bucket
    auto for_lines = [&](auto &&fn) {
        for (uint32_t c = w; c < d.nc; c += G) {
            const uint32_t L0 = c * TV16_CHUNK;
            const uint32_t nl = d.nb > L0 ? std::min(TV16_CHUNK, d.nb - L0) : 0u;
            for (uint32_t i0 = 0; i0 < nl; i0 += 64) fn(L0 + i0 + lane, L0 + i0 + lane < L0 + nl, c);
        }
    };
    for_lines([&](uint32_t li, bool ok, uint32_t) {
        if (ok) d.sums_g[li] = lane_line_sum(d.src + (size_t)li * 16);
    });
    vm_drain();
    auto get_sum = [&](uint32_t li) -> float { return d.sums_g[li]; };
    const uint32_t tailpos = d.nb * 16;
    const uint32_t ut = f2u(tail_key);
    bool tail_left = (flags & DEC_TAIL) != 0;  // the ragged tail competes and is not yet emitted
    uint32_t ub = tb;                          // keys u < ub are not yet emitted
    uint32_t left = M;                         // full lines still to emit
    uint32_t eoff = cnt;                       // output offset of the next piece
    for (uint32_t piece = 0;; ++piece) {
        // a later piece reuses the level histograms (zeroed by the previous
        // piece after its last read), the candidate buffer and the tie counts
        if (piece) C.grid_sync();
        const uint32_t nbase = uni(ld_acq_relaxed(&bc->cand_n));
        const uint32_t need = std::min(left, CAND_CAP - 1u);
        const uint32_t hi0 = ub ? ub - 1u : 0u;  // largest remaining key
        uint32_t mode = 1, blo = ub, ustar = 0, greater = 0, ties_n = 0, lvl = 0;
        bool final = true;
        if (need > 0 && ub > 0) {
            for (uint32_t i = lane; i < HBINS; i += 64) L.hist[i] = 0;
            lds_drain();
            for_lines([&](uint32_t li, bool ok, uint32_t) {
                if (!ok) return;
                const uint32_t u = f2u(get_sum(li));
                if (u < ub) atomicAdd(&L.hist[std::min((hi0 - u) >> L1_SHIFT, HBINS - 1)], 1u);
            });
            lds_drain();
            for (uint32_t i = lane; i < HBINS; i += 64) {
                const uint32_t h = L.hist[i];
                if (h) g_add(&bc->hist[0][i], h);
            }
            C.grid_sync();
            uint32_t hi = hi0, lo = 0, s = L1_SHIFT, above = 0;
            bool ovf = true;
            constexpr uint32_t BPL = HBINS / 64;  // bins per lane
            for (;;) {
                // locate the bin holding rank `need - above` (1-based) counting down from hi
                const uint32_t want = need - above;
                uint32_t loc = 0;
                for (uint32_t jj = 0; jj < BPL; ++jj) loc += ld_acq_relaxed(&bc->hist[lvl][lane * BPL + jj]);
                const uint32_t incl = wave_incl_scan(loc);
                const uint32_t excl = incl - loc;
                const uint64_t fm = __ballot(want > excl && want <= incl);
                uint32_t bstar = 0xffffffffu, cum = 0, hb = 0;
                if (fm) {
                    const uint32_t src_lane = (uint32_t)__ffsll((long long)fm) - 1u;
                    if (lane == src_lane) {
                        uint32_t cc = excl;
                        for (uint32_t jj = 0; jj < BPL; ++jj) {
                            const uint32_t h = ld_acq_relaxed(&bc->hist[lvl][lane * BPL + jj]);
                            if (want <= cc + h) { bstar = lane * BPL + jj; cum = cc; hb = h; break; }
                            cc += h;
                        }
                    }
                    bstar = (uint32_t)__builtin_amdgcn_readlane((int)bstar, (int)src_lane);
                    cum = (uint32_t)__builtin_amdgcn_readlane((int)cum, (int)src_lane);
                    hb = (uint32_t)__builtin_amdgcn_readlane((int)hb, (int)src_lane);
                }
                if (bstar == 0xffffffffu) {  // histogram does not reach `need`: collect all
                    if (lane == 0) C.fail(FAIL_LEVELS);
                    mode = 1; blo = 0;
                    break;
                }
                if (ovf && bstar == HBINS - 1) {
                    above += cum;
                    const uint64_t width = (uint64_t)(HBINS - 1) << s;
                    if ((uint64_t)hi < width) {
                        if (lane == 0) C.fail(FAIL_LEVELS);
                        mode = 1; blo = 0;
                        break;
                    }
                    hi = hi - (uint32_t)width;
                    lo = 0;
                    s = bitlen(hi) > 10 ? bitlen(hi) - 10 : 0;
                    ovf = false;
                } else {
                    const uint32_t bhi = hi - (bstar << s);
                    const int64_t blo64 = (int64_t)hi - ((int64_t)(bstar + 1) << s) + 1;
                    const uint32_t bl = (uint32_t)std::max<int64_t>((int64_t)lo, blo64);
                    const uint32_t totc = above + cum + hb;
                    // keys in [bl, ub): the whole piece fits the rank capacity
                    if (totc + 1 <= CAND_CAP) { mode = 1; blo = bl; final = need == left; break; }
                    // one key value: the keys above it, then its ties in position order
                    if (s == 0) {
                        mode = 2; ustar = bhi; greater = above + cum; ties_n = hb;
                        final = greater + ties_n >= left;
                        break;
                    }
                    above += cum;
                    hi = bhi;
                    lo = bl;
                    s = s >= 10 ? s - 10 : 0;
                }
                if (lvl + 1 >= MAX_LEVELS) {
                    if (lane == 0) C.fail(FAIL_LEVELS);
                    mode = 1; blo = lo;
                    break;
                }
                ++lvl;
                for (uint32_t i = lane; i < HBINS; i += 64) L.hist[i] = 0;
                lds_drain();
                for_lines([&](uint32_t li, bool ok, uint32_t) {
                    if (!ok) return;
                    const uint32_t u = f2u(get_sum(li));
                    if (u < ub && u >= lo && u <= hi) atomicAdd(&L.hist[(hi - u) >> s], 1u);
                });
                lds_drain();
                for (uint32_t i = lane; i < HBINS; i += 64) {
                    const uint32_t h = L.hist[i];
                    if (h) g_add(&bc->hist[lvl][i], h);
                }
                C.grid_sync();
            }
        }

        // the ragged tail's place in this piece
        // (a negative tail key has the sign bit: u >= ub, never inside a cut)
        const bool tail_sorted = mode == 1 ? tail_left && (final || (ut >= blo && ut < ub))
                                           : tail_left && ut > ustar && ut < ub;
        const bool tail_tie = mode == 2 && tail_left && ut == ustar;
        // collect: mode 1 -> keys in [blo, ub); mode 2 -> keys in (ustar, ub);
        // one slot range per ranker; mode 2 also counts each chunk's ties at ustar
        if (need > 0 && ub > 0) {
            const uint32_t kmin = mode == 1 ? blo : ustar + 1;
            uint32_t mine = 0;
            for_lines([&](uint32_t li, bool ok, uint32_t) {
                if (!ok) return;
                const uint32_t u = f2u(get_sum(li));
                mine += u < ub && u >= kmin;
            });
            mine = uni(wave_sum(mine));
            uint32_t o = nbase;
            if (lane == 0 && mine) o = g_add(&bc->cand_n, mine);
            uint32_t base = uni(o) - nbase;
            for (uint32_t c = w; c < d.nc; c += G) {
                const uint32_t L0 = c * TV16_CHUNK;
                const uint32_t nl = d.nb > L0 ? std::min(TV16_CHUNK, d.nb - L0) : 0u;
                uint32_t ties = 0;
                for (uint32_t i0 = 0; i0 < nl; i0 += 64) {
                    const uint32_t i = i0 + lane;
                    uint32_t u = 0;
                    bool p = false;
                    if (i < nl) {
                        u = f2u(get_sum(L0 + i));
                        p = u < ub && u >= kmin;
                        ties += mode == 2 && u == ustar;
                    }
                    const uint64_t m = __ballot(p);
                    const uint32_t ex = (uint32_t)__popcll(m & below_mask(lane));
                    if (p && base + ex < CAND_CAP) st_sc1(&cand[base + ex], cand_key(u, (L0 + i) * 16));
                    base += (uint32_t)__popcll(m);
                }
                if (mode == 2) {
                    const uint32_t ct = uni(wave_sum(ties));
                    if (lane == 0) st_sc1(&C.A.desc[d.cs + c].ties, ((uint64_t)C.tag(TAG_TIE) << 32) | ct);
                }
            }
        }
        C.grid_sync();  // every append / tie count is visible; every histogram read is done
        if (mode == 2) {  // lines tied at ustar, in position order after the greater keys
            const uint32_t base = eoff + 16u * greater + (tail_sorted ? d.tl : 0u);
            uint32_t all_ties = 0;
            for (uint32_t c = lane; c < d.nc; c += 64) all_ties += (uint32_t)ld_sc1(&C.A.desc[d.cs + c].ties);
            all_ties = uni(wave_sum(all_ties));
            for (uint32_t c = w; c < d.nc; c += G) {
                uint32_t before = 0;
                for (uint32_t c2 = lane; c2 < c; c2 += 64) before += (uint32_t)ld_sc1(&C.A.desc[d.cs + c2].ties);
                uint32_t rank = uni(wave_sum(before));
                const uint32_t L0 = c * TV16_CHUNK;
                const uint32_t nl = d.nb > L0 ? std::min(TV16_CHUNK, d.nb - L0) : 0u;
                for (uint32_t i0 = 0; i0 < nl; i0 += 64) {
                    const uint32_t i = i0 + lane;
                    const bool p = i < nl && f2u(get_sum(L0 + i)) == ustar;
                    const uint64_t m = __ballot(p);
                    if (p) {
                        const uint32_t ex = (uint32_t)__popcll(m & below_mask(lane));
                        const uint64_t off = (uint64_t)base + 16ull * (rank + ex);
                        if (off < d.dst_len)
                            emit_line(d, vec, (L0 + i) * 16, (uint32_t)off,
                                      std::min<uint32_t>(16u, d.dst_len - (uint32_t)off));
                    }
                    rank += (uint32_t)__popcll(m);
                }
            }
            if (w == 0 && lane == 0 && tail_tie) {
                const uint64_t off = (uint64_t)base + 16ull * all_ties;
                if (off < d.dst_len)
                    emit_line(d, false, tailpos, (uint32_t)off, std::min<uint32_t>(d.tl, d.dst_len - (uint32_t)off));
            }
        }
        uint32_t nc_all = uni(ld_acq_relaxed(&bc->cand_n)) - nbase;
        if (nc_all > CAND_CAP) {
            if (w == 0 && lane == 0) C.fail(FAIL_CAND_OVERFLOW);
            nc_all = CAND_CAP;
        }
        rank_emit(C, C.w, C.G, d, cand, eoff, nc_all, tail_sorted && nc_all < CAND_CAP, tail_key);
        if (final) break;
        // next piece: the keys below this one's cut, after its entries
        const uint32_t lines = mode == 1 ? nc_all : greater + ties_n;
        const bool tail_out = tail_sorted || tail_tie;
        eoff += 16u * lines + (tail_out ? d.tl : 0u);
        left -= std::min(left, lines);
        if (tail_out) tail_left = false;
        ub = mode == 1 ? blo : ustar;
        {  // zero this piece's level histograms (every ranker's reads are done)
            uint32_t *z = &bc->hist[0][0];
            const uint32_t words = (lvl + 1) * HBINS;
            const uint32_t per = (words + G - 1) / G;
            const uint32_t z0 = w * per, z1 = std::min(words, z0 + per);
            for (uint32_t i = z0 + lane; i < z1; i += 64) st_sc1(z + i, 0u);
        }
        if (eoff >= d.dst_len || left == 0) break;
    }
}

// Window path, ahead of the decision.  Once every chunk of the bucket has
// counted its window list, the W listed lines are known; the ranker gathers
// the set, counting-sorts it, ranks its entries r, r + R, ... within the set
// and stages their lines in LDS -- before the bucket's regime is decided, so
// that after the decision only the output offsets remain (the batch's last
// bucket is otherwise a serial tail of three memory round trips).  Work for a
// bucket that ends in regime A, or on the rare path, is dropped.
struct WinPrep {
    uint32_t ne;  // entries prepared (0: not prepared)
    bool lines;   // their lines are staged in LDS (aligned bucket)
};

__device__ __forceinline__ void win_prepare(Ctx &C, uint32_t r, uint32_t R, const BucketDesc &d, uint32_t b,
                                            uint32_t W, WinPrep &P) {
    Lds &L = C.L;
    const uint32_t lane = flane();
    const uint32_t *ckey = reinterpret_cast<const uint32_t *>(C.cand(b));
    const uint32_t *cpos = ckey + CAND_CAP;
    const uint32_t ne = (W - r + R - 1) / R;
    if (ne > 64) return;  // more than one entry per lane: the post-decision path
    gather16(ckey, (W + 3) / 4, L.wr.key);
    for (uint32_t i = lane; i < WBINS; i += 64) L.wr.bin[i] = 0;
    lds_drain();
    constexpr uint32_t SH = 29 - 10;  // keys < 2^29
    for (uint32_t i = lane; i < W; i += 64) atomicAdd(&L.wr.bin[L.wr.key[i] >> SH], 1u);
    lds_drain();
    {  // exclusive scan of the bins, 16 per lane
        constexpr uint32_t BPL = WBINS / 64;
        uint32_t sum = 0;
        for (uint32_t q = 0; q < BPL; ++q) sum += L.wr.bin[lane * BPL + q];
        uint32_t run = wave_incl_scan(sum) - sum;
        for (uint32_t q = 0; q < BPL; ++q) {
            const uint32_t c = L.wr.bin[lane * BPL + q];
            L.wr.bin[lane * BPL + q] = run;
            run += c;
        }
    }
    lds_drain();
    for (uint32_t i = lane; i < W; i += 64) {
        const uint32_t k = L.wr.key[i];
        L.wr.srt[atomicAdd(&L.wr.bin[k >> SH], 1u)] = k;  // bin[x] ends as the end of bin x
    }
    lds_drain();
    if (lane < ne) {
        const uint32_t k = L.wr.key[r + lane * R];
        const uint32_t bn = k >> SH;
        const uint32_t lo = bn ? L.wr.bin[bn - 1] : 0u, hi = L.wr.bin[bn];
        uint32_t rank = lo;
        for (uint32_t x = lo; x < hi; ++x) rank += L.wr.srt[x] < k;
        L.wr.ent[lane] = make_uint4(rank, ld_sc1(&cpos[k & 0xfffu]), 0u, k);
    }
    lds_drain();
    P.ne = ne;
    P.lines = aligned16(d);
    if (P.lines) {  // stage the lines (a quad of lanes per entry) where the keys were
        float4 *lines = reinterpret_cast<float4 *>(L.wr.key);
        const uint32_t c4 = 4 * (lane & 3);
        float4 x[4];
#pragma unroll
        for (uint32_t g0 = 0; g0 < 4; ++g0) {
            const uint32_t el = g0 * 16 + (lane >> 2);
            x[g0] = el < ne ? *reinterpret_cast<const float4 *>(d.src + (size_t)L.wr.ent[el].y + c4)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (uint32_t g0 = 0; g0 < 4; ++g0) lines[(g0 * 16 + (lane >> 2)) * 4 + (lane & 3)] = x[g0];
        lds_drain();
    }
}

// Window path after the decision, for a prepared ranker: offsets from the
// bucket's count, the ragged tail (set index W) inserted into the order when it
// competes, and the stores.
__device__ __forceinline__ void win_emit(Ctx &C, uint32_t r, uint32_t R, const BucketDesc &d, uint32_t cnt, uint32_t W,
                                         bool tail, float tail_key, uint32_t tb, const WinPrep &P) {
    Lds &L = C.L;
    const uint32_t lane = flane();
    constexpr uint32_t SH = 29 - 10;
    const uint32_t wlo = tb > WIN ? tb - WIN : 0u;
    const uint32_t ut = f2u(tail_key);  // a negative tail key has the sign bit: never in the window
    const bool tail_in = tail && ut >= wlo && ut < tb && W < CAND_CAP;
    const uint32_t tail_k = ((tb - 1u - ut) << 12) | W;
    const uint32_t tailpos = d.nb * 16;
    const uint32_t c4 = 4 * (lane & 3);
    const float4 *lines = reinterpret_cast<const float4 *>(L.wr.key);
#pragma unroll
    for (uint32_t g0 = 0; g0 < 4; ++g0) {
        const uint32_t el = g0 * 16 + (lane >> 2);
        if (el >= P.ne) break;
        const uint4 en = L.wr.ent[el];
        const bool tb4 = tail_in && tail_k < en.w;  // the tail sorts before this entry
        const uint64_t off = (uint64_t)cnt + 16ull * (en.x + (tb4 ? 1u : 0u)) - (tb4 ? (uint64_t)(16u - d.tl) : 0ull);
        if (off >= d.dst_len) continue;
        const uint32_t len = std::min<uint32_t>(16u, d.dst_len - (uint32_t)off);
        const uint32_t bi = en.y + c4 + (uint32_t)d.idx_offset;
        if (P.lines && len == 16) {
            *reinterpret_cast<float4 *>(d.val + off + c4) = lines[el * 4 + (lane & 3)];
            *reinterpret_cast<uint4 *>(d.idx + off + c4) = make_uint4(bi, bi + 1, bi + 2, bi + 3);
        } else {
            for (uint32_t cc = 0; cc < 4; ++cc) {
                if (c4 + cc < len) {
                    d.val[off + c4 + cc] = d.src[(size_t)en.y + c4 + cc];
                    d.idx[off + c4 + cc] = bi + cc;
                }
            }
        }
    }
    if (tail_in && W % R == r) {  // the tail is this ranker's entry: its rank among the set
        const uint32_t bn = tail_k >> SH;
        const uint32_t lo = bn ? L.wr.bin[bn - 1] : 0u, hi = L.wr.bin[bn];
        uint32_t less = 0;
        for (uint32_t x = lo + lane; x < hi; x += 64) less += L.wr.srt[x] < tail_k;
        const uint32_t rank = lo + uni(wave_sum(less));
        const uint64_t off = (uint64_t)cnt + 16ull * rank;
        if (off < d.dst_len) {
            const uint32_t len = std::min<uint32_t>(d.tl, d.dst_len - (uint32_t)off);
            if (lane < len) {
                d.val[off + lane] = d.src[(size_t)tailpos + lane];
                d.idx[off + lane] = tailpos + lane + (uint32_t)d.idx_offset;
            }
        }
    }
}

// The heap fill of bucket b, run by every ranker once the bucket's decision
// is posted (the window path's group prepares ahead of it).
template <int STAGE>
__device__ __forceinline__ void rank_bucket(Ctx &C, uint32_t b) {
    const BucketDesc &d = C.A.bk[b];
    const uint32_t lane = flane();
    // RK rankers per bucket on the window path (a rotating group, so the set
    // is fetched RK times rather than G times)
    const uint32_t NG = std::max(1u, C.G / RK);
    const uint32_t g = b % NG;
    const bool grp = C.w % NG == g;
    const uint32_t R = (C.G - g + NG - 1) / NG, r = C.w / NG;
    WinPrep P{0, false};
    uint32_t W = 0;
    if (grp && STAGE != 5) {
        // the group's first ranker alone polls the finishers' list counter
        // (polling a line under atomic adds slows the adds), then posts the
        // bucket's window-line count for the others
        ReadyLine &RL = C.ctl()->ready[b];
        const uint32_t tR = C.tag(TAG_RDY);
        uint64_t st7 = 0;
        if (r == 0) {
            uint32_t ch = 0, wl = 0;
            for (uint32_t spins = 0;; ++spins) {
                ch = 0;
                wl = 0;
                for (uint32_t i = lane; i < C.G; i += 64) {
                    const uint64_t v = ld_sc1(&C.ctl()->lst[i].w[b]);
                    if ((uint32_t)(v >> 32) == C.tag(TAG_LST)) {
                        ch += ((uint32_t)v >> 16) & 0xffffu;
                        const uint32_t x = (uint32_t)v & 0xffffu;
                        wl += x == 0xffffu ? CAND_CAP : x;  // saturated: too many for the window path
                    }
                }
                ch = uni(wave_sum(ch));
                wl = uni(wave_sum(wl));
                if (ch >= d.nc) break;
                __builtin_amdgcn_s_sleep(STG_TV16_DEC_SLEEP);
                if (spin_expired(spins, st7)) { if (lane == 0) C.spin_fail(5, b, ch, d.nc); return; }
            }
            W = std::min(wl, CAND_CAP);
            if (lane == 0) st_sc1(&RL.w, ((uint64_t)tR << 32) | W);
        } else {
            uint64_t rw = ld_sc1(&RL.w);
            for (uint32_t spins = 0; (uint32_t)(rw >> 32) != tR; ++spins) {
                __builtin_amdgcn_s_sleep(STG_TV16_DEC_SLEEP);
                rw = ld_sc1(&RL.w);
                if (spin_expired(spins, st7)) { if (lane == 0) C.spin_fail(5, b, 0, d.nc); return; }
            }
            W = uni((uint32_t)rw);
        }
        if (b < 16) C.stamp(64 + 4 * b + 1, 0);
        if (W > 0 && W + 1 <= CAND_CAP && r < W) win_prepare(C, r, R, d, b, W, P);
    }
    Decision &D = C.ctl()->dec[b];
    const uint32_t tD = C.tag(TAG_DEC);
    uint64_t w0 = ld_sc1(&D.w[0]);
    uint64_t st6 = 0;
    for (uint32_t spins = 0; (uint32_t)(w0 >> 32) != tD; ++spins) {
        __builtin_amdgcn_s_sleep(STG_TV16_DEC_SLEEP);
        w0 = ld_sc1(&D.w[0]);
        if (spin_expired(spins, st6)) { if (lane == 0) C.spin_fail(4, b, (uint32_t)(w0 >> 32), tD); return; }
    }
    const uint32_t flags = uni((uint32_t)w0);
    if (!(flags & DEC_B)) return;
    const uint64_t w1 = ld_sc1(&D.w[1]), w2 = ld_sc1(&D.w[2]), w3 = ld_sc1(&D.w[3]);
    const uint32_t cnt = uni((uint32_t)(w1 >> 32)), M = uni((uint32_t)w1);
    const uint32_t Wtot = uni((uint32_t)(w2 >> 32));
    const float tail_key = __uint_as_float(uni((uint32_t)w2));
    const float t = __uint_as_float(uni((uint32_t)w3));
    if (b < 16) C.stamp(64 + 4 * b, 0);
    if (flags & DEC_WIN) {
        // the window holds the top M: every chunk wrote its window lines at
        // its exchanged offset (all counted before W was read)
        const bool tail = (flags & DEC_TAIL) != 0;
        if (!grp || r >= Wtot + (tail ? 1u : 0u)) return;
        if (P.ne && W == Wtot) {
            win_emit(C, r, R, d, cnt, Wtot, tail, tail_key, f2u(t), P);
        } else {
            // (the ready line said every list was counted)
            rank_window(C, r, R, d, b, cnt, Wtot, tail, tail_key, f2u(t));
        }
    } else {
        rank_rare(C, b, flags, cnt, M, t, tail_key);
    }
    if (b < 16) C.stamp(64 + 4 * b + 2, 0);
}

// STAGE (diagnostics only, STG_DEBUG_TV16_STAGE): 0 = full codec; 1 = the
// streaming waves' work only (the finisher releases buffers at once);
// 3 = plain streaming read (calibration); 4 = full codec + s_memrealtime
// stamps (tools/stamps.py); 5 = full codec without the regime-B heap fill.
template <int STAGE, bool EF>
__global__ void __launch_bounds__(FWG, 8) tv16_batch(BatchArgs A) {
    __shared__ Lds L;
    Ctx C{A, L, gridDim.x, blockIdx.x, 0, A.ctl, A.cand, A.fail, STAGE == 4};
    if (STAGE == 4 && threadIdx.x < 128) L.stamp[threadIdx.x] = 0;
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
    if (threadIdx.x < MAX_BATCH) { L.pw[threadIdx.x] = 0; L.cum[threadIdx.x] = 0; }
    if (threadIdx.x == 0) {
        L.fdone = 0;
        // slots 0 and 1: chunks w and G + w; later slots take the next chunks
        // of the call's counter (2G + n, taken by the finisher), so every
        // workgroup's slots hold increasing chunks and chunks are taken in order
        L.cid[0] = C.w;
        L.cid[1] = C.G + C.w;
        for (uint32_t i = 0; i < CIDR; ++i) { L.cok[i] = 0; L.mid[i] = 0; }
        L.cok[0] = 1;
        L.cok[1] = 2;
    }
    __syncthreads();
    const uint32_t wave = (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave < NS) {
        for (uint32_t j = 0;; ++j) {
            uint64_t st8 = 0;
            uint32_t spins = 0;
            for (; lds_ld(&L.cok[j % CIDR]) != j + 1; ++spins) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, st8)) { if (flane() == 0) C.spin_fail(6, j, lds_ld(&L.cok[j % CIDR]), wave); break; }
            }
            if (C.stamping && spins && flane() == 0) atomicAdd(&L.stamp[121], spins);
            const uint32_t k = uni(lds_ld(&L.cid[j % CIDR]));
            if (k >= A.K) break;
            asm volatile("" : "+s"(C.w), "+s"(C.G));
            scan_chunk<STAGE, EF>(C, j, k, wave);
        }
    } else if (wave == FIN) {
        if (STG_TV16_PRIO) __builtin_amdgcn_s_setprio(3);  // short bursts issue ahead of the streaming waves
        FinState F{0};
        for (uint32_t j = 0;; ++j) {
            uint64_t st9 = 0;
            for (uint32_t spins = 0; lds_ld(&L.cok[j % CIDR]) != j + 1; ++spins) {
                __builtin_amdgcn_s_sleep(1);
                if (spin_expired(spins, st9)) { if (flane() == 0) C.spin_fail(7, j, lds_ld(&L.cok[j % CIDR]), 99); break; }
            }
            const uint32_t k = uni(lds_ld(&L.cid[j % CIDR]));
            if (k >= A.K) break;
            asm volatile("" : "+s"(C.w), "+s"(C.G), "+s"(C.ctlp), "+s"(C.candp), "+s"(C.failp));
            finish_chunk<STAGE>(C, j, k, F);
        }
        vm_drain();
        flush_lists(C, F);
    } else {
        if (STG_TV16_PRIO) __builtin_amdgcn_s_setprio(2);
        if (STAGE != 1 && STAGE != 3) {
            for (uint32_t b = 0; b < A.nbk; ++b) {
                asm volatile("" : "+s"(C.w), "+s"(C.G), "+s"(C.ctlp), "+s"(C.candp), "+s"(C.failp));
                rank_bucket<STAGE>(C, b);
            }
        }
        if (STAGE == 4) {
            // the finisher and streamers are done with their stamps when every
            // bucket is decided; the ranker flushes them last
            for (uint32_t i = flane(); i < 128; i += 64) A.stamps[C.w * 128 + i] = L.stamp[i];
        }
    }
}

}  // namespace

hipError_t launch_tv16(const Tv16Launch &a, const DevWS &ws, hipStream_t s) {
    if (!a.nb) return hipSuccess;
    if (a.nb > MAX_BATCH || !a.epoch || a.epoch >= (1u << 24)) return hipErrorInvalidValue;
    BatchArgs A{};
    uint32_t K = 0;
    for (uint32_t i = 0; i < a.nb; ++i) {
        const Tv16Bucket &b = a.b[i];
        if (b.first) {  // first threshold from sequential line sums (thresholdv16.cpp:36-54)
            const uint32_t nblk = (uint32_t)((b.n + 15) / 16);
            tv16_seq_sums<<<(nblk + STG_WG - 1) / STG_WG, STG_WG, 0, s>>>(b.src, b.n, b.sums, nblk);
            const uint32_t bk = std::min<uint32_t>(b.k / 16, nblk - 1);
            hipError_t e = launch_radix_select(b.sums, nblk, 0xffffffffu, 0, nullptr, bk, ws, a.num_cu, s);
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
        d.cs = K;
        d.nc = std::max<uint32_t>(1, (d.nb + TV16_CHUNK - 1) / TV16_CHUNK);
        K += d.nc;
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
    A.stamps = a.b[a.nb - 1].count_out + 1;  // STAGE 4: words after the last bucket's count
    // this launch's share of the device's two 1024-thread workgroups per CU
    // (all of them for one stream; launches from several streams split them),
    // all co-resident for the in-launch exchanges; no more than there are chunks
    const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(std::min<uint32_t>(a.max_wg, K), MAXG));
    static const int dbg_stage = getenv("STG_DEBUG_TV16_STAGE") ? atoi(getenv("STG_DEBUG_TV16_STAGE")) : 0;
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    switch (dbg_stage) {
        case 1: tv16_batch<1, false><<<G, FWG, 0, s>>>(A); break;
        case 3: tv16_batch<3, false><<<G, FWG, 0, s>>>(A); break;
        case 4: tv16_batch<4, false><<<G, FWG, 0, s>>>(A); break;
        case 5: tv16_batch<5, false><<<G, FWG, 0, s>>>(A); break;
        default:
            if (ef) tv16_batch<0, true><<<G, FWG, 0, s>>>(A);
            else tv16_batch<0, false><<<G, FWG, 0, s>>>(A);
            break;
    }
    if (a.ev) {
        (void)hipEventRecord(a.ev[1], s);
        (void)hipEventRecord(a.ev[2], s);
    }
    return hipGetLastError();
}

}  // namespace stg
