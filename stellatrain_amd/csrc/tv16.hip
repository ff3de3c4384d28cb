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
// One persistent launch per batch of buckets (tv16_batch): 1024-thread
// workgroups (1 or 2 per CU, all co-resident), each owning a contiguous range
// of every bucket's lines.  Per bucket b:
//   scan(b)   stream the range once (a quad of lanes per line, DPP cross-lane
//             adds in the AVX tree order), keep the line sums in LDS, stage the
//             qualifying lines' data in LDS, count S >= t and the lines in a
//             window just below t; publish both counts as tagged granules;
//   finish(b) gather every workgroup's granules (one wave, all loads in
//             flight), derive the regime, emit this range's qualifying lines
//             with global rank < kb (+1 partial) from LDS; workgroup 0 writes
//             the tail, the AIMD threshold and the count; regime B only: rank
//             the window candidates (or run a radix descent when the window
//             does not hold them) with last-arriver grid barriers and emit the
//             heap fill in (sum desc, position asc) order.
// The launch runs scan(b+1) before finish(b): bucket b's count exchange and
// the streaming tail of its slowest workgroups hide behind the next bucket's
// streaming pass.  A key's first call runs tv16_seq_sums + a radix select
// (select.hip) before the launch.
#include <algorithm>
#include <cstdlib>

#include "ws.h"

namespace stg {

namespace {

typedef unsigned int u4v __attribute__((ext_vector_type(4)));

constexpr uint32_t FWG = 1024;     // workgroup: 16 waves
constexpr uint32_t FNW = FWG / 64;
constexpr uint32_t L1_SHIFT = 14;  // level-1 bin width in ulps below t (~0.2% of t)
constexpr uint32_t LA = 2;         // pipeline lookahead: finish(b) runs after scan(b + LA)
constexpr uint32_t NBUF = LA + 1;  // LDS buffer sets (line sums, staged lines) in flight
constexpr uint32_t LINES_B = 2048; // line sums kept in LDS per workgroup and buffer set
constexpr uint32_t STAGE_B = 88;   // qualifying lines staged in LDS per workgroup and buffer set
constexpr uint32_t SCAN_U = 8;     // float4 per lane per load batch
constexpr uint32_t MAX_J = LINES_B / FWG;
constexpr uint32_t WIN = 1u << 17; // regime-B window below t, in ulps (~1.6% of t)

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
    float *sums_g;  // line sums of ranges beyond LINES_B
    uint32_t nb, tl, dst_len;
    int32_t idx_offset;
    uint32_t per, rem;  // line ranges: workgroup w owns per + (w < rem) lines
    uint32_t pad[2];
};

struct BatchArgs {
    BucketDesc bk[MAX_BATCH];
    uint32_t nbk;
    uint32_t epoch;  // 1 .. 2^24-1
    FillCtl *ctl;
    uint64_t *cand;
    uint32_t *fail;
    uint32_t *stamps;  // STAGE 4 diagnostics only
};

// LDS of one workgroup (< 80 KiB: two workgroups per CU).
struct Lds {
    float sum[NBUF][LINES_B];       // line sums, by buffer set (bucket % NBUF)
    float4 stage[NBUF][STAGE_B * 4];  // staged qualifying lines (64 B each)
    uint32_t stage_line[NBUF][STAGE_B];
    union {
        uint64_t cand[CAND_CAP];    // regime-B candidates (rank phase)
        uint4 pf[MAX_FILL_WG];      // previous bucket's granules (scan -> finish)
    };
    uint64_t mask[MAX_J * FNW];
    uint32_t hist[HBINS];
    uint32_t wt[MAX_J * FNW + 1];
    uint32_t sh[FNW + 1];
    uint64_t sh64[FNW];
    uint32_t dec[8];
    uint32_t xch[FNW][4];           // count exchange partials per polling wave
    uint32_t nst[NBUF];
    uint32_t stamp[32];             // STAGE 4: timestamps, flushed at kernel end
    uint32_t cnt[2 * FNW];          // per-wave counts of a scan
};

// Per-bucket values a workgroup carries from scan(b) to finish(b).
struct Carry {
    float t, inc;
    uint32_t qw, ww;  // this range's qualifying / window line counts
};

// Granules of the previous bucket, loaded (per lane of the gather waves) at
// the start of the next bucket's scan so the exchange round trip overlaps the
// streaming pass; finish() re-polls only lanes whose tag was not yet current.
struct Prefetch {};  // (kept in LDS: Lds::pf, filled by LDS-DMA)

__device__ __forceinline__ uint32_t bitlen(uint32_t x) { return x ? 32u - __clz(x) : 0u; }

// Workgroup-uniform values read from memory or LDS: move them to SGPRs (the
// compiler cannot prove uniformity; VGPR copies would spill at 64 VGPRs, and
// a scratch reload waits for every outstanding store of the wave).
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ float uni(float x) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x))); }

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

struct Ctx {
    const BatchArgs &A;
    Lds &L;
    uint32_t G, w, wave;
    uint32_t nbar;  // grid-barrier rounds used so far (the same in every workgroup)
    bool probe;     // STAGE 4: sub-phase stamps of the probed bucket

    // STAGE 4 only: stamps[16*1024 + w*16 + k]
    __device__ __forceinline__ void sub(uint32_t k) const {
        if (probe && ftid() == 0) L.stamp[16 + k] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    }

    __device__ __forceinline__ uint32_t tag(uint32_t b) const { return (A.epoch << 8) | b; }
    // Fresh (opaque) thread / lane ids per phase: keeps the compiler from
    // hoisting per-thread addresses of every phase out of the bucket loop into
    // live registers (they would spill).
    __device__ __forceinline__ uint32_t ftid() const {
        uint32_t x = threadIdx.x;
        asm volatile("" : "+v"(x));
        return x;
    }
    FillCtl *ctlp;    // control pointers, laundered per bucket iteration
    uint64_t *candp;
    uint32_t *failp;
    __device__ __forceinline__ FillCtl *ctl() const { return ctlp; }
    __device__ __forceinline__ uint64_t *cand() const { return candp; }
    __device__ __forceinline__ uint32_t *fail() const { return failp; }
    __device__ __forceinline__ uint32_t flane() const {
        uint32_t x;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(x));
        return x;
    }
    // Workgroup w's line range of a bucket (host-computed split, scalar math).
    __device__ __forceinline__ uint32_t range_lo(const BucketDesc &d) const {
        return w * d.per + (w < d.rem ? w : d.rem);
    }
    __device__ __forceinline__ uint32_t range_len(const BucketDesc &d) const { return d.per + (w < d.rem ? 1u : 0u); }

    // Last-arriver grid barrier: the workgroup whose arrival completes round r
    // writes every workgroup's own go word; each workgroup polls only its own.
    __device__ __forceinline__ void grid_sync() {
        const uint32_t r = ++nbar;
        FillCtl *fc = ctl();
        CallCtl *cc = &fc->cc[A.epoch & 1u];
        const uint64_t go = ((uint64_t)(A.epoch << 8) << 32) | r;
        const uint32_t tid = ftid();
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) L.dec[7] = __hip_atomic_fetch_add(&cc->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (L.dec[7] == r * G - 1) {
            for (uint32_t i = tid; i < G; i += FWG) st_sc1(&fc->slot[i].go, go);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (tid == 0) {
            for (uint32_t spins = 0; ld_sc1(&fc->slot[w].go) != go; ++spins) {
                __builtin_amdgcn_s_sleep(1);
                if (spins > (1u << 24)) { atomicOr(fail(), (uint32_t)FAIL_SPIN_TIMEOUT); break; }
            }
        }
        __syncthreads();
    }
};

// ---- scan(b): stream this workgroup's range of bucket b ----
template <int STAGE, bool LDS_SUMS>
__device__ __forceinline__ Carry scan_bucket(Ctx &C, uint32_t b, Prefetch &pf) {
    const BucketDesc &d = C.A.bk[b];
    Lds &L = C.L;
    if (b >= LA && C.wave * 64 < C.G) {
        // The previous bucket's granules, fetched global -> LDS (no registers)
        // as the oldest load of this scan, so the exchange round trip overlaps
        // the streaming pass; finish() re-polls only stale lanes.
        const uint32_t v = C.wave * 64 + C.flane();
        const uint64_t *src = &C.ctl()->gran[b - LA][v < C.G ? v : 0][0];
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(src), &L.pf[C.wave * 64], 16, 0,
                                         16 /* sc1 */);
    }
    const uint32_t par = b % NBUF;
    const uint32_t L0 = C.range_lo(d), nl = C.range_len(d);
    Carry cr;
    // Read before publishing this bucket's counts: workgroup 0 rewrites the
    // state only after it has seen every workgroup's counts.
    cr.t = uni(d.state->t);
    cr.inc = uni(d.state->inc);
    const float t = cr.t;
    const uint32_t tb = f2u(t);
    const uint32_t wlo = tb > WIN ? tb - WIN : 0u;  // window [wlo, tb) just below t
    if (C.ftid() == 0) L.nst[par] = 0;
    __syncthreads();

    const uint32_t lane = C.flane(), wave = C.wave, q = lane & 3;
    const uint32_t lane_line = wave * 16 + (lane >> 2);  // line of this lane in a step
    constexpr uint32_t STEP = FWG / 4;                   // lines per step
    const uint32_t nbatch = ((nl + STEP - 1) / STEP + SCAN_U - 1) / SCAN_U;
    uint32_t cnt_w = 0, win_w = 0;
    // One batch of SCAN_U float4 per lane in flight; the 32 waves per CU
    // supply the memory-level parallelism (tools/ubench_stream.hip: 1 x 1024
    // threads/CU stream at ~4.0 TB/s, 2 x 1024 at ~5.4-5.8, nontemporal loads
    // +5%).  Buffer loads (nt) through a descriptor bounded to the range: one
    // 32-bit voffset per lane, the step in soffset, and lanes past the range
    // read zeros from the hardware bounds check (no clamping code).
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(d.src + (size_t)L0 * 16), 0, nl * 64u, 0x00020000);
    const uint32_t voff0 = lane_line * 64u + q * 16u;
    for (uint32_t bt = 0; bt < nbatch; ++bt) {
        // opaque per batch: keeps the compiler from hoisting SCAN_U line
        // indices into live registers across the loop (they would spill)
        uint32_t ll = lane_line;
        asm volatile("" : "+v"(ll));
        float4 v[SCAN_U];
#pragma unroll
        for (uint32_t u = 0; u < SCAN_U; ++u) {
            const u4v t4 = __builtin_amdgcn_raw_buffer_load_b128(
                rsrc, voff0, (int)((bt * SCAN_U + u) * STEP * 64u), 2 /* nt */);
            v[u] = make_float4(__uint_as_float(t4.x), __uint_as_float(t4.y), __uint_as_float(t4.z),
                               __uint_as_float(t4.w));
        }
#pragma unroll
        for (uint32_t u = 0; u < SCAN_U; ++u) {
            const uint32_t i = (bt * SCAN_U + u) * STEP + ll;
            if (STAGE == 3) {
                cnt_w += f2u(v[u].x + v[u].y + v[u].z + v[u].w) == 0x7f800001u;
                continue;
            }
            const float S = quad_line_sum(v[u]);  // the same in all four lanes of the quad
            const bool in = i < nl;
            if (in && q == 0) {
                if (LDS_SUMS) L.sum[par][i] = S;
                else d.sums_g[L0 + i] = S;
            }
            const uint32_t us = f2u(S);
            const bool qual = in && S >= t;
            const uint64_t bq = __ballot(qual && q == 0);
            win_w += (uint32_t)__popcll(__ballot(in && q == 0 && us >= wlo && us < tb));
            if (bq) {  // stage the qualifying lines (all four lanes of each quad)
                cnt_w += (uint32_t)__popcll(bq);
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&L.nst[par], (uint32_t)__popcll(bq));
                base = __builtin_amdgcn_readfirstlane(base);
                if (qual) {
                    // qualifying quads before this one: bq has bits only at quad
                    // leaders (multiples of 4), so leader p < this leader iff
                    // p + 3 < lane -- a lane-count of bq << 3 (scalar shift)
                    const uint64_t b3 = bq << 3;
                    const uint32_t slot = base + __builtin_amdgcn_mbcnt_hi(
                        (uint32_t)(b3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b3, 0u));
                    if (slot < STAGE_B) {
                        // lane-in-quad recomputed here (a live copy would spill)
                        uint32_t lq;
                        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lq));
                        lq &= 3u;
                        L.stage[par][slot * 4 + lq] = v[u];
                        if (lq == 0) L.stage_line[par][slot] = i;
                    }
                }
            }
        }
    }
    if (lane == 0) { L.cnt[wave] = cnt_w; L.cnt[FNW + wave] = win_w; }
    __syncthreads();
    cr.qw = cr.ww = 0;
#pragma unroll
    for (uint32_t i = 0; i < FNW; ++i) { cr.qw += L.cnt[i]; cr.ww += L.cnt[FNW + i]; }
    // workgroup-uniform: keep the carry in SGPRs across the next scan
    cr.qw = __builtin_amdgcn_readfirstlane(cr.qw);
    cr.ww = __builtin_amdgcn_readfirstlane(cr.ww);
    if (STAGE == 1 || STAGE == 3) {
        if (cnt_w == 12345u) d.count_out[1] = win_w;  // keep the loop alive
        return cr;
    }
    // published by the last wave: a wave's scratch reload or vmcnt(0) waits
    // for its own outstanding stores, and the gather waves are the first ones
    if (C.ftid() == FWG - 64) {
        const uint64_t tg = (uint64_t)C.tag(b) << 32;
        st_sc1(&C.ctl()->gran[b][C.w][0], tg | cr.qw);
        st_sc1(&C.ctl()->gran[b][C.w][1], tg | cr.ww);
    }
    return cr;
}

// Mode-1 / mode-2 follow-up state of a regime-B bucket.
struct Defer {
    uint32_t active, b, cnt;
    uint32_t nc;         // candidate count (window path) or ~0 = read cand_n
    uint32_t tail_cand;  // the ragged tail competes in the heap fill
    float tail_key;
};

// Distributed rank-and-emit of a collected candidate set: output order is
// (sum desc, position asc) = ascending composite key (~ord(sum) << 32 | pos);
// an entry's rank is the number of smaller keys, counted by one wave per
// entry over the LDS copy of the set (+ the ragged tail when it competes).
__device__ __forceinline__ void rank_emit(Ctx &C, const BucketDesc &d, const uint64_t *cand, uint32_t cnt,
                                          uint32_t nc_all, bool add_tail, float tail_key) {
    Lds &L = C.L;
    const uint32_t total = nc_all + (add_tail ? 1u : 0u);
    const uint32_t first_e = C.w * FNW;  // entries handled here: e = w*FNW + wave + k*G*FNW
    if (first_e >= total) return;
    const uint32_t tailpos = d.nb * 16;
    const uint64_t tail_comp = ((uint64_t)(~ford(tail_key)) << 32) | (uint64_t)tailpos;
    for (uint32_t i = C.ftid(); i < total; i += FWG) L.cand[i] = i < nc_all ? ld_sc1(&cand[i]) : tail_comp;
    __syncthreads();
    for (uint32_t e = first_e + C.wave; e < total; e += C.G * FNW) {
        const uint64_t key = L.cand[e];
        uint32_t less = 0;
        for (uint32_t j = C.flane(); j < total; j += 64) less += L.cand[j] < key;
        const uint32_t rank = wave_sum(less);
        const bool is_tail = add_tail && key == tail_comp;
        const bool tail_before = add_tail && tail_comp < key;
        const uint32_t pos = (uint32_t)key;
        const uint32_t len = is_tail ? d.tl : 16u;
        const uint64_t off = (uint64_t)cnt + 16ull * rank - (tail_before ? (uint64_t)(16u - d.tl) : 0ull);
        if (off < d.dst_len) {
            const uint32_t Ln = std::min<uint32_t>(len, d.dst_len - (uint32_t)off);
            if (C.flane() < Ln) {
                d.val[off + C.flane()] = d.src[(size_t)pos + C.flane()];
                d.idx[off + C.flane()] = pos + C.flane() + (uint32_t)d.idx_offset;
            }
        }
    }
    __syncthreads();  // L.cand is reused
}

// ---- finish(b): exchange, regime, emission, AIMD; regime B heap fill ----
template <int STAGE>
__device__ __forceinline__ Defer finish_bucket(Ctx &C, uint32_t b, const Carry &cr, const Prefetch &pf) {
    const BucketDesc &d = C.A.bk[b];
    Lds &L = C.L;
    FillCtl *ctl = C.ctl();
    const uint32_t par = b % NBUF;
    const uint32_t G = C.G, w = C.w, tid = C.ftid(), lane = C.flane(), wave = C.wave;
    const uint32_t L0 = C.range_lo(d), nl = C.range_len(d);
    const bool lds_sums = nl <= LINES_B;
    const bool vec = ((reinterpret_cast<uintptr_t>(d.src) | reinterpret_cast<uintptr_t>(d.idx) |
                       reinterpret_cast<uintptr_t>(d.val)) & 15u) == 0;
    auto get_sum = [&](uint32_t i) -> float { return lds_sums ? L.sum[par][i] : d.sums_g[L0 + i]; };
    const float t = cr.t, inc = cr.inc;
    const uint32_t tb = f2u(t);
    const uint32_t wlo = tb > WIN ? tb - WIN : 0u;
    const uint32_t kb = d.dst_len / 16, r = d.dst_len % 16;
    auto bc = [&]() { return &C.ctl()->cc[C.A.epoch & 1u].bk[b]; };  // per use: not held live
    uint64_t *cand = C.cand() + (size_t)(b & 3u) * CAND_CAP;

    C.sub(1);
    // ---- count exchange: wave j gathers workgroups [64j, 64j+64) (one
    //      granule pair per lane, all in flight), re-polling only stale ones ----
    const uint32_t nsw = (G + 63) / 64;
    if (wave < nsw) {
        const uint32_t tg = C.tag(b);
        const uint32_t v = wave * 64 + lane;
        const uint4 e = L.pf[v];  // prefetched during this bucket's successor's scan
        uint64_t g = ((uint64_t)e.y << 32) | e.x, g2 = ((uint64_t)e.w << 32) | e.z;
        bool pend = v < G && ((uint32_t)(g >> 32) != tg || (uint32_t)(g2 >> 32) != tg);
        if (C.probe && lane == 0) atomicAdd(&L.stamp[16 + 8], (uint32_t)__popcll(__ballot(pend)));
        uint32_t polls = 0;
        for (uint32_t spins = 0;; ++spins) {
            if (!__any(pend)) break;
            ++polls;
            if (pend) {
                g = ld_sc1(&ctl->gran[b][v][0]);
                g2 = ld_sc1(&ctl->gran[b][v][1]);
                pend = (uint32_t)(g >> 32) != tg || (uint32_t)(g2 >> 32) != tg;
            }
            if (!__any(pend)) break;
            __builtin_amdgcn_s_sleep(1);
            if (spins > (1u << 22)) { atomicOr(C.fail(), (uint32_t)FAIL_SPIN_TIMEOUT); break; }
        }
        if (C.probe && lane == 0) atomicMax(&L.stamp[16 + 9], polls);
        const uint32_t c = v < G ? (uint32_t)g : 0u, cw = v < G ? (uint32_t)g2 : 0u;
        const uint32_t tot = wave_sum(c), wtot = wave_sum(cw);
        const uint32_t bef = wave_sum(v < w ? c : 0u), wbef = wave_sum(v < w ? cw : 0u);
        if (lane == 0) {
            L.xch[wave][0] = bef;
            L.xch[wave][1] = tot;
            L.xch[wave][2] = wbef;
            L.xch[wave][3] = wtot;
        }
    }
    __syncthreads();
    uint32_t P = 0, Qtot = 0, Wbef = 0, Wtot = 0;
    for (uint32_t j = 0; j < nsw; ++j) {
        P += L.xch[j][0];
        Qtot += L.xch[j][1];
        Wbef += L.xch[j][2];
        Wtot += L.xch[j][3];
    }
    P = uni(P);
    Qtot = uni(Qtot);
    Wbef = uni(Wbef);
    Wtot = uni(Wtot);
    __syncthreads();
    if (STAGE == 2) return Defer{};

    C.sub(2);
    // ---- regime (identical in every workgroup) ----
    const uint32_t lim = kb + (r ? 1u : 0u);
    const uint32_t c0 = Qtot >= lim ? d.dst_len : 16u * Qtot;
    bool tail_cand = false;
    float tail_key = 0.f;
    uint32_t ct = 0;
    if (c0 < d.dst_len && d.tl) {
        const float *tp = d.src + (size_t)d.nb * 16;
        float s = 0.f;
        for (uint32_t i = 0; i < d.tl; ++i) s += tp[i];
        s = uni(s);
        if (s * 16.0f >= t * (float)d.tl) ct = std::min(d.dst_len - c0, d.tl);
        else { tail_cand = true; tail_key = s * 16.0f / (float)d.tl; }
    }
    const uint32_t cnt = c0 + ct;
    const bool regimeB = cnt < d.dst_len;

    // ---- ordered emission of this range's qualifying lines ----
    // In-range rank of line i = j*FWG + tid via ballot masks (order j, wave, lane).
    if (P < lim && cr.qw) {
        const uint32_t nj = (nl + FWG - 1) / FWG;
        if (nj <= MAX_J && cr.qw <= STAGE_B) {
            // every qualifying line is staged in LDS: one thread per staged line
            for (uint32_t j = 0; j < nj; ++j) {
                const uint32_t i = j * FWG + tid;
                const uint64_t bal = __ballot(i < nl && get_sum(i) >= t);
                if (lane == 0) { L.mask[j * FNW + wave] = bal; L.wt[j * FNW + wave] = (uint32_t)__popcll(bal); }
            }
            __syncthreads();
            if (tid == 0) {
                uint32_t acc = 0;
                for (uint32_t i = 0; i < nj * FNW; ++i) { const uint32_t x = L.wt[i]; L.wt[i] = acc; acc += x; }
            }
            __syncthreads();
            for (uint32_t e = tid; e < cr.qw; e += FWG) {
                const uint32_t i = L.stage_line[par][e];
                const uint32_t grp = (i / FWG) * FNW + ((i % FWG) >> 6), ln = i & 63;
                const uint64_t m = L.mask[grp];
                const uint32_t g = P + L.wt[grp] + (uint32_t)__popcll(m & (ln ? (~0ull >> (64 - ln)) : 0ull));
                if (g < lim) {
                    const uint32_t pos = (L0 + i) * 16;
                    const uint32_t len = g == kb ? r : 16u;
                    const uint32_t off = 16 * g;
                    if (vec && len == 16) {
                        float4 *v4 = reinterpret_cast<float4 *>(d.val + off);
                        uint4 *i4 = reinterpret_cast<uint4 *>(d.idx + off);
                        const uint32_t bi = pos + (uint32_t)d.idx_offset;
#pragma unroll
                        for (uint32_t c = 0; c < 4; ++c) {
                            v4[c] = L.stage[par][e * 4 + c];
                            i4[c] = make_uint4(bi + 4 * c, bi + 4 * c + 1, bi + 4 * c + 2, bi + 4 * c + 3);
                        }
                    } else {
                        const float *sv = reinterpret_cast<const float *>(&L.stage[par][e * 4]);
                        for (uint32_t c = 0; c < len; ++c) {
                            d.val[off + c] = sv[c];
                            d.idx[off + c] = pos + c + (uint32_t)d.idx_offset;
                        }
                    }
                }
            }
            __syncthreads();
        } else {
            // staging overflowed (low threshold) or a long range: re-read src
            const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
            uint32_t base = P;
            for (uint32_t j0 = 0; j0 < nj && base < lim; j0 += MAX_J) {
                const uint32_t jn = std::min(nj - j0, MAX_J);
                uint32_t flags = 0;
                for (uint32_t j = 0; j < jn; ++j) {
                    const uint32_t i = (j0 + j) * FWG + tid;
                    const bool f = i < nl && get_sum(i) >= t;
                    flags |= (uint32_t)f << j;
                    const uint64_t bal = __ballot(f);
                    if (lane == 0) L.wt[j * FNW + wave] = (uint32_t)__popcll(bal);
                }
                __syncthreads();
                if (tid == 0) {
                    uint32_t acc = 0;
                    for (uint32_t i = 0; i < jn * FNW; ++i) { const uint32_t x = L.wt[i]; L.wt[i] = acc; acc += x; }
                    L.wt[MAX_J * FNW] = acc;
                }
                __syncthreads();
                for (uint32_t j = 0; j < jn; ++j) {
                    const uint64_t bal = __ballot((flags >> j) & 1u);
                    if ((flags >> j) & 1u) {
                        const uint32_t g = base + L.wt[j * FNW + wave] + (uint32_t)__popcll(bal & lt);
                        if (g < lim) {
                            const uint32_t line = L0 + (j0 + j) * FWG + tid;
                            emit_line(d, vec, line * 16, 16 * g, g == kb ? r : 16u);
                        }
                    }
                }
                base += L.wt[MAX_J * FNW];
                __syncthreads();
            }
        }
    }

    C.sub(3);
    // ---- tail, AIMD, count (workgroup 0) ----
    if (w == 0 && tid == 0) {
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
    C.sub(4);
    if (!regimeB || STAGE == 5) return Defer{};

    // ---- heap fill = top candidates by (sum desc, position asc) ----
    const uint32_t rem = d.dst_len - cnt;
    const uint32_t ncand = d.nb - Qtot;  // non-qualifying full lines
    const uint32_t M = std::min((rem + 15u) / 16u, ncand);
    const uint32_t hi0 = tb - 1u;        // largest candidate key (keys u < tb)

    // mode 1: collect keys >= blo; mode 2: ties at ustar taken in position order
    uint32_t mode = 1, blo = tb, ustar = 0, greater = 0;
    const bool win_ok = M > 0 && Wtot >= M && Wtot + 1 <= CAND_CAP;
    if (win_ok) {
        blo = wlo;  // the window holds the top M: no histogram needed
    } else if (M > 0) {
        for (uint32_t i = tid; i < HBINS; i += FWG) L.hist[i] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < nl; i += FWG) {
            const uint32_t u = f2u(get_sum(i));
            if (u < tb) atomicAdd(&L.hist[std::min((hi0 - u) >> L1_SHIFT, HBINS - 1)], 1u);
        }
        __syncthreads();
        for (uint32_t i = tid; i < HBINS; i += FWG)
            if (L.hist[i]) atomicAdd(&bc()->hist[0][i], L.hist[i]);
        C.grid_sync();
        uint32_t lvl = 0, hi = hi0, lo = 0, s = L1_SHIFT, above = 0;
        bool ovf = true;
        for (;;) {
            // locate the bin holding rank `need` (1-based) counting down from hi
            const uint32_t need = M - above;
            const uint32_t cbin = tid < HBINS ? ld_acq_relaxed(&bc()->hist[lvl][tid]) : 0u;
            uint32_t total;
            const uint32_t before = blk_excl_scan<FNW>(cbin, L.sh, &total);
            if (tid == 0) { L.dec[2] = 0xffffffffu; L.dec[3] = 0; L.dec[4] = 0; }
            __syncthreads();
            if (tid < HBINS && need > before && need <= before + cbin) { L.dec[2] = tid; L.dec[3] = before; L.dec[4] = cbin; }
            __syncthreads();
            const uint32_t bstar = uni(L.dec[2]), cum = uni(L.dec[3]), hb = uni(L.dec[4]);
            __syncthreads();
            if (bstar == 0xffffffffu) {  // histogram does not reach `need`: collect all
                if (tid == 0) atomicOr(C.fail(), (uint32_t)FAIL_LEVELS);
                mode = 1; blo = 0;
                break;
            }
            if (ovf && bstar == HBINS - 1) {
                above += cum;
                const uint64_t width = (uint64_t)(HBINS - 1) << s;
                if ((uint64_t)hi < width) {
                    if (tid == 0) atomicOr(C.fail(), (uint32_t)FAIL_LEVELS);
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
                if (totc + 1 <= CAND_CAP) { mode = 1; blo = bl; break; }
                if (s == 0) { mode = 2; ustar = bhi; greater = above + cum; break; }
                above += cum;
                hi = bhi;
                lo = bl;
                s = s >= 10 ? s - 10 : 0;
            }
            if (++lvl >= MAX_LEVELS) {
                if (tid == 0) atomicOr(C.fail(), (uint32_t)FAIL_LEVELS);
                mode = 1; blo = lo;
                break;
            }
            for (uint32_t i = tid; i < HBINS; i += FWG) L.hist[i] = 0;
            __syncthreads();
            for (uint32_t i = tid; i < nl; i += FWG) {
                const uint32_t u = f2u(get_sum(i));
                if (u < tb && u >= lo && u <= hi) atomicAdd(&L.hist[(hi - u) >> s], 1u);
            }
            __syncthreads();
            for (uint32_t i = tid; i < HBINS; i += FWG)
                if (L.hist[i]) atomicAdd(&bc()->hist[lvl][i], L.hist[i]);
            C.grid_sync();
        }
    }

    const uint32_t tailpos = d.nb * 16;
    const bool tail_in_greater = tail_cand && mode == 2 && tail_key > u2f(ustar);
    // collect (write-through): mode 1 -> keys in [blo, tb); mode 2 -> keys in (ustar, tb).
    // The window path knows every workgroup's slot range from the exchanged
    // window counts (no atomics); the rare histogram paths append with one
    // atomic per workgroup and step.
    if (M > 0) {
        const uint32_t kmin = mode == 1 ? blo : ustar + 1;
        uint32_t mine = 0, run = Wbef;
        for (uint32_t i0 = 0; i0 < nl; i0 += FWG) {
            const uint32_t i = i0 + tid;
            uint32_t u = 0;
            bool p = false;
            if (i < nl) {
                u = f2u(get_sum(i));
                p = u < tb && u >= kmin;
                mine += mode == 2 && u == ustar;
            }
            uint32_t n_here;
            const uint32_t ex = blk_excl_scan<FNW>((uint32_t)p, L.sh, &n_here);
            if (!n_here) continue;
            uint32_t base;
            if (win_ok) {
                base = run;
                run += n_here;
            } else {
                if (tid == 0) L.dec[7] = atomicAdd(&bc()->cand_n, n_here);
                __syncthreads();
                base = L.dec[7];
                __syncthreads();
            }
            if (p && base + ex < CAND_CAP)
                st_sc1(&cand[base + ex], ((uint64_t)(~(u | 0x80000000u)) << 32) | (uint64_t)((L0 + i) * 16));
        }
        if (mode == 2) {
            const uint32_t my_ties = (uint32_t)blk_sum64<FNW>(mine, L.sh64);
            if (tid == 0) st_sc1(&ctl->wg_ties[b & 3u][w], my_ties);
        }
    }
    C.sub(5);
    if (mode == 1) {
        // The common case: publish "candidates written" and rank the set
        // after the next bucket's scan (rank_deferred), when every workgroup's
        // candidates are long in place -- no grid barrier on the critical path.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) st_sc1(&ctl->cdone[b][w], (uint64_t)C.tag(b) << 32);
        Defer D;
        D.active = 1;
        D.b = b;
        D.cnt = cnt;
        D.nc = win_ok ? Wtot : 0xffffffffu;
        D.tail_cand = tail_cand ? 1u : 0u;
        D.tail_key = tail_key;
        return D;
    }
    C.grid_sync();  // every append / tie count is visible
    {  // mode 2: lines tied at ustar, in position order after the greater keys
        uint64_t pb = 0, pt = 0;
        for (uint32_t i = tid; i < G; i += FWG) {
            const uint32_t x = ld_acq_relaxed(&ctl->wg_ties[b & 3u][i]);
            pt += x;
            if (i < w) pb += x;
        }
        uint32_t rank = (uint32_t)blk_sum64<FNW>(pb, L.sh64);
        const uint32_t all_ties = (uint32_t)blk_sum64<FNW>(pt, L.sh64);
        const uint32_t base = cnt + 16u * greater + (tail_in_greater ? d.tl : 0u);
        for (uint32_t i0 = 0; i0 < nl; i0 += FWG) {
            const uint32_t i = i0 + tid;
            const bool p = i < nl && f2u(get_sum(i)) == ustar;
            uint32_t n_here;
            const uint32_t ex = blk_excl_scan<FNW>((uint32_t)p, L.sh, &n_here);
            if (p) {
                const uint64_t off = (uint64_t)base + 16ull * (rank + ex);
                if (off < d.dst_len)
                    emit_line(d, vec, (L0 + i) * 16, (uint32_t)off, std::min<uint32_t>(16u, d.dst_len - (uint32_t)off));
            }
            rank += n_here;
        }
        if (w == 0 && tid == 0 && tail_cand && tail_key == u2f(ustar)) {
            const uint64_t off = (uint64_t)base + 16ull * all_ties;
            if (off < d.dst_len)
                emit_line(d, false, tailpos, (uint32_t)off, std::min<uint32_t>(d.tl, d.dst_len - (uint32_t)off));
        }
    }
    uint32_t nc_all = uni(ld_acq_relaxed(&bc()->cand_n));
    if (nc_all > CAND_CAP) {
        if (w == 0 && tid == 0) atomicOr(C.fail(), (uint32_t)FAIL_CAND_OVERFLOW);
        nc_all = CAND_CAP;
    }
    rank_emit(C, d, cand, cnt, nc_all, tail_in_greater && nc_all < CAND_CAP, tail_key);
    return Defer{};
}

// Deferred rank-and-emit of a mode-1 candidate set (bucket D.b), run one
// bucket later.  Workgroups with no entries to rank return at once when the
// set size is known (window path); the others wait for every workgroup's
// "candidates written" tag (normally already set) and rank.
__device__ __forceinline__ void rank_deferred(Ctx &C, const Defer &D) {
    if (!D.active) return;
    const BucketDesc &d = C.A.bk[D.b];
    const uint32_t first_e = C.w * FNW;
    if (D.nc != 0xffffffffu && first_e >= D.nc + (D.tail_cand && D.nc < CAND_CAP ? 1u : 0u)) return;
    Lds &L = C.L;
    const uint32_t nsw = (C.G + 63) / 64;
    if (C.wave < nsw) {
        const uint32_t tg = C.tag(D.b);
        const uint32_t v = C.wave * 64 + C.flane();
        bool pend = v < C.G;
        for (uint32_t spins = 0;; ++spins) {
            if (pend) pend = (uint32_t)(ld_sc1(&C.ctl()->cdone[D.b][v]) >> 32) != tg;
            if (!__any(pend)) break;
            __builtin_amdgcn_s_sleep(2);
            if (spins > (1u << 22)) { atomicOr(C.fail(), (uint32_t)FAIL_SPIN_TIMEOUT); break; }
        }
    }
    __syncthreads();
    uint32_t nc_all = D.nc;
    if (nc_all == 0xffffffffu) nc_all = uni(ld_acq_relaxed(&C.ctl()->cc[C.A.epoch & 1u].bk[D.b].cand_n));
    if (nc_all > CAND_CAP) {
        if (C.ftid() == 0) atomicOr(C.fail(), (uint32_t)FAIL_CAND_OVERFLOW);
        nc_all = CAND_CAP;
    }
    (void)L;
    rank_emit(C, d, C.cand() + (size_t)(D.b & 3u) * CAND_CAP, D.cnt, nc_all, D.tail_cand && nc_all < CAND_CAP,
              D.tail_key);
}

// STAGE (diagnostics only, STG_DEBUG_TV16_STAGE): 0 = full codec; 1 = return
// after the streaming passes; 2 = skip everything after the count exchanges;
// 3 = plain streaming read (calibration); 4 = full codec + per-workgroup
// s_memrealtime stamps: stamps[w*16 + 15] at start, [w*16 + 2b] after scan(b),
// [w*16 + 2b + 1] after finish(b) and the deferred rank of b-1 (b < 7),
// [w*16 + 14] = XCC id; 5 = full codec without the regime-B heap fill.
template <int STAGE>
__global__ void __launch_bounds__(FWG, 8) tv16_batch(BatchArgs A) {
    __shared__ Lds L;
    Ctx C{A, L, gridDim.x, blockIdx.x, (uint32_t)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), 0,
          false, A.ctl, A.cand, A.fail};
    // STAGE 4: stamps go to LDS (a global store here would make the wave's
    // next vmcnt wait include its write-back) and are flushed at the end
    auto stamp = [&](uint32_t k) {
        if (STAGE == 4 && C.ftid() == 0 && k < 16) L.stamp[k] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    };
    if (STAGE == 4 && C.ftid() < 32) L.stamp[C.ftid()] = 0;
    stamp(15);
    if (STAGE == 4 && C.ftid() == 0) L.stamp[14] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));
    {  // zero the next call's per-call counters (this call never touches them)
        uint32_t *z = reinterpret_cast<uint32_t *>(&A.ctl->cc[(A.epoch + 1) & 1u]);
        constexpr uint32_t words = sizeof(CallCtl) / 4;
        const uint32_t per = (words + C.G - 1) / C.G;
        const uint32_t z0 = C.w * per, z1 = std::min(words, z0 + per);
        for (uint32_t i = z0 + C.ftid(); i < z1; i += FWG) st_sc1(z + i, 0u);
    }
    // software pipeline: scan(b) | finish(b-LA) | deferred rank of b-LA-1
    static_assert(LA == 2, "carry rotation below is written for LA == 2");
    Carry ca{}, cb{}, cur{};  // scan results of buckets b-2, b-1, b (no indexed locals: no scratch)
    Defer pend{};             // regime-B set awaiting its rank-and-emit
    Prefetch pf{};            // granules of bucket b-LA, loaded during scan(b) (into Lds::pf)
    for (uint32_t b = 0; b <= A.nbk + LA; ++b) {
        // opaque per iteration: addresses derived from the workgroup id are
        // recomputed (scalar) instead of hoisted into live vector registers
        asm volatile("" : "+s"(C.w), "+s"(C.G), "+s"(C.ctlp), "+s"(C.candp), "+s"(C.failp));
        if (b < A.nbk) {
            // ranges beyond LINES_B keep their line sums in global scratch
            if (C.range_len(A.bk[b]) <= LINES_B) cur = scan_bucket<STAGE, true>(C, b, pf);
            else cur = scan_bucket<STAGE, false>(C, b, pf);
            if (b < 7) stamp(2 * b);
        }
        if (STAGE == 1 || STAGE == 3) continue;
        Defer dn{};
        C.probe = STAGE == 4 && b == 2 + LA;
        if (b >= LA && b - LA < A.nbk) dn = finish_bucket<STAGE>(C, b - LA, ca, pf);
        C.sub(6);
        rank_deferred(C, pend);
        C.sub(7);
        C.probe = false;
        if (b >= LA && b - LA < 7) stamp(2 * (b - LA) + 1);
        pend = dn;
        ca = cb;
        cb = cur;
    }
    if (STAGE == 4) {
        __syncthreads();
        if (C.ftid() < 16) A.stamps[C.w * 16 + C.ftid()] = L.stamp[C.ftid()];
        else if (C.ftid() < 32) A.stamps[16 * 1024 + C.w * 16 + C.ftid() - 16] = L.stamp[C.ftid()];
    }
}

}  // namespace

hipError_t launch_tv16(const Tv16Launch &a, const DevWS &ws, hipStream_t s) {
    if (!a.nb) return hipSuccess;
    if (a.nb > MAX_BATCH || !a.epoch || a.epoch >= (1u << 24)) return hipErrorInvalidValue;
    BatchArgs A{};
    uint32_t max_nb = 1;
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
        d.nb = (uint32_t)(b.n / 16);
        d.tl = (uint32_t)(b.n % 16);
        d.dst_len = b.dst_len;
        d.idx_offset = b.idx_offset;
        max_nb = std::max(max_nb, d.nb);
    }
    A.nbk = a.nb;
    A.epoch = a.epoch;
    A.ctl = ws.ctl;
    A.cand = ws.cand;
    A.fail = ws.fail;
    A.stamps = a.b[a.nb - 1].count_out + 1;  // STAGE 4: words after the last bucket's count
    // wg_per_cu 1024-thread workgroups per CU (2: 32 waves, full occupancy for
    // one stream; 1: two launches from two streams share the CUs), all
    // co-resident for the in-launch exchanges, >= 1024 lines of the largest
    // bucket each
    const uint32_t G = std::max<uint32_t>(
        1, std::min<uint32_t>(std::min<uint32_t>(a.wg_per_cu * (uint32_t)a.num_cu, (max_nb + 1023) / 1024),
                              MAX_FILL_WG));
    for (uint32_t i = 0; i < a.nb; ++i) {
        A.bk[i].per = A.bk[i].nb / G;
        A.bk[i].rem = A.bk[i].nb % G;
    }
    static const int dbg_stage = getenv("STG_DEBUG_TV16_STAGE") ? atoi(getenv("STG_DEBUG_TV16_STAGE")) : 0;
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    switch (dbg_stage) {
        case 1: tv16_batch<1><<<G, FWG, 0, s>>>(A); break;
        case 2: tv16_batch<2><<<G, FWG, 0, s>>>(A); break;
        case 3: tv16_batch<3><<<G, FWG, 0, s>>>(A); break;
        case 4: tv16_batch<4><<<G, FWG, 0, s>>>(A); break;
        case 5: tv16_batch<5><<<G, FWG, 0, s>>>(A); break;
        default: tv16_batch<0><<<G, FWG, 0, s>>>(A); break;
    }
    if (a.ev) {
        (void)hipEventRecord(a.ev[1], s);
        (void)hipEventRecord(a.ev[2], s);
    }
    return hipGetLastError();
}

}  // namespace stg
