// tv16lone.hip -- thresholdv16's one-bucket scan on gfx950.
//
// Reference: ThresholdvCompressor16::impl_simd_v2 stages 1-2
// (/root/reference/backend/src/compress/thresholdv16.cpp:138-205), the line
// sum hsum_float_avx (:57-73).  The engine compresses one bucket per call
// (engine/modules/compress.cpp:141): a lone 64 MiB bucket is 2048 chunks of
// 512 lines (32 KiB), one per 256-thread workgroup, eight per CU.
//
// The batched scan (tv16.hip) orders its emission inside the launch: each
// chunk waits for the counts of the chunks before it, so chunks are taken
// from a ticket counter in order -- 512 tickets on one word at the start of a
// lone launch cost ~6 us (~88 per us), and the last chunk's look-back, the
// regime decision and the emission all sit at the launch's end.  Here no
// workgroup ever waits on another: chunk c goes to workgroup c mod G, and
// each chunk leaves only its lists --
//   ldesc[c] = {qualifying lines, window lines}       (true counts)
//   lq[c][r] = the r-th qualifying line of the chunk   (line within the chunk;
//              the call's tag, low 16 bits, above it: the finish's freshness check)
//   lv[c][r] = its 16 floats (staged from the stream: the finish never re-reads them)
//   lw[c][r] = {sum bits, line | qualifying lines before it << 16} of its r-th
//              window line (sum in [t - 2^18 ulps, t), thresholdv16 regime B)
// -- and the fill launch that follows (tv16fill.hip, lfin mode) takes the
// prefixes, decides the regime, emits the qualifying lines in index order and
// orders the regime-B fill.  A chunk with more lines than its lists hold is
// re-read there.
//
// Per workgroup NW waves; wave s streams lines (s + NW m) * 16 + lane / 4 of
// the chunk, a quad of lanes per line (a float4 each, DPP adds in the AVX tree
// order), D float4 loads in flight per lane through a buffer descriptor
// bounded to the chunk.  The lists of a chunk are built in LDS (two slots: a
// workgroup with several chunks streams the next while the last wave done
// with one sorts and writes its lists).
#include <algorithm>
#include <cstdlib>

#include "tv16_dev.h"

namespace stg {

namespace {

using namespace tv16;

constexpr uint32_t kEfAux = 2;  // cache policy of the fused residual stores (2: nontemporal)


static_assert(LCHUNK <= 512 && LMAXC <= 4096 && LQCAP < 1024, "binned entry packing: chunk:12 | line:9 | qb:10");
static_assert(LNBIN << 8 == TV16_WIN, "bins of 256 ulps cover the window");

struct LLds {
    float4 qv[2][LQCAP][4];  // their data (a float4 per lane of the line's quad)
    uint32_t ql[2][LQCAP];  // qualifying lines of the chunk in the slot (unordered)
    uint64_t wl[2][LWCAP];  // window lines: sum bits << 32 | line
    uint32_t qn[2], wn[2], done[2], fin[2];
};

// A slot's lists, ordered, to global memory: by the last wave done with the
// chunk.  Ranks by counting (a few dozen entries per chunk at k = 1 %).  Its
// window lines also go to their bins (ws.h LNBIN): the bin's count is taken
// first, so the atomic's round trip overlaps the list writes.
__device__ __forceinline__ void finalize(LLds &L, const LScanArgs &A, uint32_t sl, uint32_t c, uint32_t j,
                                         uint32_t tb) {
    const uint32_t lane = flane();
    const uint32_t qn = uni(lds_ld(&L.qn[sl])), wn = uni(lds_ld(&L.wn[sl]));
    const uint32_t ql = std::min(qn, LQCAP), wlc = std::min(wn, LWCAP);
    static_assert(LWCAP <= 64, "one window entry per lane");
    const uint64_t we = lane < wlc ? L.wl[sl][lane] : ~0ull;
    uint32_t wbin = 0, wslot = LBCAP;
    if (lane < wlc) {
        wbin = (tb - 1u - (uint32_t)(we >> 32)) >> 8;  // < LNBIN: the sum is in [t - 2^18 ulps, t)
        wslot = g_add(&A.whist[whist_word(wbin)], 1u);
    }
    uint32_t *lq = A.lq + (size_t)c * LQCAP;
    uint2 *lw = A.lw + (size_t)c * LWCAP;
    float4 *lv = A.lv + (size_t)c * LQCAP * 4;
    // lq, lv, went and the counts are read inside this launch by the finish
    // (tv16lf2.h): written through (sc1), as the hand-off requires
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(lq, 0, LQCAP * 4u, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(lv, 0, LQCAP * 64u, 0x00020000);
    const __amdgpu_buffer_rsrc_t re = __builtin_amdgcn_make_buffer_rsrc(A.went, 0, LNBIN * LBCAP * 8u, 0x00020000);
    const uint32_t qtag = (A.tag ^ (A.skip == 5 ? 1u : 0u)) << 16;  // (STG_LF2_SKIP=5: a wrong tag, the check's test)
    // entry e of the list has rank r_e; its line data (four float4) goes to
    // lv[r_e]: lane = 16 entries x 4 quarters per round
    for (uint32_t e0 = 0; e0 < ql; e0 += 16) {
        const uint32_t e = e0 + (lane >> 2), qq = lane & 3u;
        if (e < ql) {
            const uint32_t li = L.ql[sl][e];
            uint32_t r = 0;
            for (uint32_t x = 0; x < ql; ++x) r += L.ql[sl][x] < li;
            if (qq == 0) __builtin_amdgcn_raw_buffer_store_b32(li | qtag, rq, r * 4u, 0, 16 /* sc1 */);
            const float4 x = L.qv[sl][e][qq];
            u4v t4;
            t4.x = __float_as_uint(x.x); t4.y = __float_as_uint(x.y); t4.z = __float_as_uint(x.z); t4.w = __float_as_uint(x.w);
            __builtin_amdgcn_raw_buffer_store_b128(t4, rv, (r * 4u + qq) * 16u, 0, 16 /* sc1 */);
        }
    }
    if (wlc) {  // at most one entry per lane
        const uint32_t li = (uint32_t)we;
        uint32_t r = 0, qb = 0;
        for (uint32_t x = 0; x < wlc; ++x) r += (uint32_t)L.wl[sl][x] < li;
        for (uint32_t x = 0; x < ql; ++x) qb += L.ql[sl][x] < li;
        if (lane < wlc) {
            st_sc1(reinterpret_cast<uint64_t *>(lw + r), (uint64_t)(li | qb << 16) << 32 | (uint32_t)(we >> 32));
            if (wslot < LBCAP) {
                typedef unsigned int u2v __attribute__((ext_vector_type(2)));
                u2v t2;
                t2.x = (uint32_t)(we >> 32);
                t2.y = c << 19 | li << 10 | qb;
                __builtin_amdgcn_raw_buffer_store_b64(t2, re, (wbin * LBCAP + wslot) * 8u, 0, 16 /* sc1 */);
            }
        }
    }
    // the chunk's counts, tagged with the call: the finish (tv16lf2.h) waits
    // for every chunk's tag; the lists above are drained first
    vm_drain();
    if (lane == 0) st_sc1(reinterpret_cast<uint64_t *>(A.ldesc) + c, (uint64_t)A.tag << 32 | wn << 16 | qn);
    lds_drain();
    if (lane == 0) {
        L.qn[sl] = 0;
        L.wn[sl] = 0;
        L.done[sl] = 0;
    }
    lds_drain();
    if (lane == 0) lds_st(&L.fin[sl], j + 1);
}

// GS > 0: the gather-add fused into the stream (gather.hip, ModuleCpuGather::run,
// engine/modules/cpu_gather.cpp:59-87): up to GS more input streams (the
// residual, then grad[1] .. grad[N-1]) are read beside the bucket, summed into
// it in gather.hip's order, and the sum is stored back once (grad[0] ends as
// the gather-add leaves it) and is what the line sums see.
#include "tv16lf2.h"

union LScanLds {
    LLds s;
    Lf2Lds f;
};
static_assert(sizeof(LScanLds) <= 160 * 1024 / 8, "eight scan workgroups per CU");

// Eight waves per SIMD (64 VGPRs) for the plain and error-feedback scans, whose
// finish (tv16lf2.h) would otherwise set the register budget; the gather
// scans keep theirs (their finish is the fill launch's).
template <bool EF, uint32_t NW, uint32_t D, uint32_t GS>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(GS ? 1 : 8, 8))) tv16_lscan(LScanArgs A) {
    __shared__ LScanLds U;
    LLds &L = U.s;
    const uint32_t tid = threadIdx.x;
    if (tid < 2) { L.qn[tid] = 0; L.wn[tid] = 0; L.done[tid] = 0; L.fin[tid] = 0; }
    // the extra streams in summation order: the residual, then grad[1] ..
    const uint32_t ns = GS ? (A.gres ? 1u : 0u) + (A.gn ? A.gn - 1u : 0u) : 0u;
    auto xs = [&](uint32_t e) -> const float * {
        if (A.gres) return e == 0 ? A.gres : A.gsrc[e];
        return A.gsrc[e + 1u];
    };
    if (GS && blockIdx.x == 0 && tid < A.tl) {  // the ragged tail (the stream covers full lines)
        const size_t e = (size_t)A.nb * 16 + tid;
        float acc = A.src[e];
        for (uint32_t x = 0; x < ns; ++x) acc += xs(x)[e];
        st_sc1(reinterpret_cast<uint32_t *>(const_cast<float *>(A.src)) + e, f2u(acc));  // (read by the finish: sc1)
    }
    // the next call's counters (the finish of this call uses the other copy)
    if (blockIdx.x == 0 && tid < sizeof(CallCtl) / 4) st_sc1(A.zero_next + tid, 0u);
    if (blockIdx.x == 0 && A.whist_next)  // the next call's window histogram
        for (uint32_t i = tid; i < LNBIN; i += NW * 64) st_sc1(A.whist_next + i, 0u);
    const uint32_t s = uni(tid >> 6), lane = flane(), q = lane & 3u;
    const uint32_t lane_line = s * 16 + (lane >> 2);
    float t = 0.f, inc0 = 0.f;
    uint32_t tb = 0, wlo = 0;
    for (uint32_t j = 0;; ++j) {
        const uint32_t c = blockIdx.x + j * gridDim.x;
        if (c >= A.nc) break;
        const uint32_t sl = j & 1u;
        if (j >= 2) {  // the slot's previous chunk (j - 2) has been written out (its finalizing wave is running)
            uint64_t st0 = 0;
            for (uint32_t spins = 0; lds_ld(&L.fin[sl]) < j - 1; ++spins) {
                __builtin_amdgcn_s_sleep(1);
                // intra-workgroup (the finalizing wave runs): a timeout means a
                // broken wave, and the slot may still be in use, so the call
                // is marked failed (poisoned count, failure word) before the
                // wave goes on and its lists can no longer be trusted
                if (spin_expired(spins, st0)) {
                    if (lane == 0) { g_or(A.fail, FAIL_SPIN_TIMEOUT); st_sc1(A.count_out, POISON_COUNT); }
                    break;
                }
            }
        }
        const uint32_t L0 = c * LCHUNK;
        const uint32_t nl = A.nb > L0 ? std::min(LCHUNK, A.nb - L0) : 0u;
        const uint32_t steps = (nl + 15) / 16;
        const uint32_t mine = steps > s ? (steps - s + NW - 1) / NW : 0u;
        const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float *>(A.src + (size_t)L0 * 16), 0, nl * 64u, 0x00020000);
        const __amdgpu_buffer_rsrc_t rsrc_r = __builtin_amdgcn_make_buffer_rsrc(
            EF ? A.resid + (size_t)L0 * 16 : nullptr, 0, (EF && A.resid) ? nl * 64u : 0u, 0x00020000);
        auto load = [&](uint32_t m) -> float4 {
            uint32_t voff = lane_line * 64u + q * 16u;
            asm volatile("" : "+v"(voff));  // opaque: no hoisted per-step offsets
            const u4v t4 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff + m * (NW * 1024u), 0, 2 /* nt */);
            return make_float4(__uint_as_float(t4.x), __uint_as_float(t4.y), __uint_as_float(t4.z),
                               __uint_as_float(t4.w));
        };
        __amdgpu_buffer_rsrc_t rx[GS ? GS : 1];  // extra streams (past ns: no records, reads 0, never added)
#pragma unroll
        for (uint32_t e = 0; e < (GS ? GS : 1u); ++e)
            rx[e] = __builtin_amdgcn_make_buffer_rsrc(e < ns ? const_cast<float *>(xs(e)) + (size_t)L0 * 16 : nullptr, 0,
                                                      e < ns ? nl * 64u : 0u, 0x00020000);
        auto load_x = [&](uint32_t e, uint32_t m) -> float4 {
            uint32_t voff = lane_line * 64u + q * 16u;
            asm volatile("" : "+v"(voff));
            const u4v t4 = __builtin_amdgcn_raw_buffer_load_b128(rx[e], voff + m * (NW * 1024u), 0, 2 /* nt */);
            return make_float4(__uint_as_float(t4.x), __uint_as_float(t4.y), __uint_as_float(t4.z),
                               __uint_as_float(t4.w));
        };
        auto store_s = [&](uint32_t m, float4 x) {  // the gathered sum back into the bucket
            uint32_t voff = lane_line * 64u + q * 16u;
            asm volatile("" : "+v"(voff));
            u4v t4;
            t4.x = __float_as_uint(x.x); t4.y = __float_as_uint(x.y); t4.z = __float_as_uint(x.z); t4.w = __float_as_uint(x.w);
            // written through: the finish in this launch reads popped lines
            // from the bucket (sc1 loads) once the chunk is listed
            __builtin_amdgcn_raw_buffer_store_b128(t4, rsrc, voff + m * (NW * 1024u), 0, 16 /* sc1 */);
        };
        auto store_r = [&](uint32_t m, float4 x) {
            uint32_t voff = lane_line * 64u + q * 16u;
            asm volatile("" : "+v"(voff));
            u4v t4;
            t4.x = __float_as_uint(x.x); t4.y = __float_as_uint(x.y); t4.z = __float_as_uint(x.z); t4.w = __float_as_uint(x.w);
            __builtin_amdgcn_raw_buffer_store_b128(t4, rsrc_r, voff + m * (NW * 1024u), 0, kEfAux);
        };
        float4 v[D], w[GS ? GS : 1][D];
#pragma unroll
        for (uint32_t u = 0; u < D; ++u) {
            v[u] = load(u);
#pragma unroll
            for (uint32_t e = 0; e < GS; ++e) w[e][u] = load_x(e, u);
        }
        if (STG_LF2_STAMPS && j == 0 && blockIdx.x == 0 && tid == 0) A.dbg[0] = (uint32_t)__builtin_amdgcn_s_memrealtime();
        if (j == 0) {  // the threshold, read while the chunk's first loads are in flight
            t = uni(A.state->t);
            inc0 = uni(A.state->inc);
            if (blockIdx.x == 0 && tid == 0) {  // the finish decides with the threshold the scan used
                st_sc1(reinterpret_cast<uint32_t *>(&A.cp->t), f2u(t));
                st_sc1(reinterpret_cast<uint32_t *>(&A.cp->inc), f2u(A.state->inc));
            }
            tb = f2u(t);
            wlo = tb > TV16_WIN ? tb - TV16_WIN : 0u;  // window [wlo, tb) just below t
            __syncthreads();  // the slot counters are zeroed
        }
        for (uint32_t m0 = 0; m0 < mine; m0 += D) {
#pragma unroll
            for (uint32_t u = 0; u < D; ++u) {
                float4 x = v[u];
                if (GS) {  // dst + residual + grad[1] + ... in gather.hip's order
#pragma unroll
                    for (uint32_t e = 0; e < GS; ++e) {
                        const float4 y = w[e][u];
                        const bool on = e < ns;
                        x.x = on ? x.x + y.x : x.x;
                        x.y = on ? x.y + y.y : x.y;
                        x.z = on ? x.z + y.z : x.z;
                        x.w = on ? x.w + y.w : x.w;
                        w[e][u] = load_x(e, m0 + u + D);
                    }
                    store_s(m0 + u, x);
                }
                uint32_t ll = lane_line;
                asm volatile("" : "+v"(ll));
                const uint32_t i = (m0 + u) * (NW * 16u) + ll;  // line within the chunk
                const float S = quad_line_sum(x);  // the same in all four lanes of the quad
                if (EF) store_r(m0 + u, x);
                v[u] = load(m0 + u + D);
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
                if (bw) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&L.wn[sl], (uint32_t)__popcll(bw));
                    base = __builtin_amdgcn_readfirstlane(base);
                    if (win && q == 0) {
                        const uint32_t slot = base + (uint32_t)__popcll(bw & below_mask(lane));
                        if (slot < LWCAP) L.wl[sl][slot] = ((uint64_t)us << 32) | i;
                    }
                }
                if (bq) {
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&L.qn[sl], (uint32_t)__popcll(bq));
                    base = __builtin_amdgcn_readfirstlane(base);
                    if (qual) {  // every lane of the quad stages its quarter of the line
                        // quads before this one: bq has bits only at quad leaders,
                        // so leader p < this leader iff p + 3 < lane
                        const uint64_t b3 = bq << 3;
                        const uint32_t slot = base + __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(b3 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b3, 0u));
                        if (slot < LQCAP) {
                            L.qv[sl][slot][q] = x;
                            if (q == 0) L.ql[sl][slot] = i;
                        }
                    }
                }
            }
        }
        lds_drain();
        if (GS) vm_drain();  // the gathered sums stored before the chunk's counts are (the finish reads them)
        uint32_t old = 0;
        if (lane == 0) old = atomicAdd(&L.done[sl], 1u);
        if (uni(old) == NW - 1) {  // every other wave's list adds were drained first
            finalize(L, A, sl, c, j, tb);
        }
    }
    if (A.fin && blockIdx.x + A.fin >= gridDim.x)
        lf2_finish(U.f, A, blockIdx.x + A.fin - gridDim.x, t, inc0);
}

}  // namespace

hipError_t launch_tv16_lscan(LScanArgs &a, int num_cu, hipStream_t s) {
    if (!a.nc) { a.fin = 0; return hipSuccess; }
    // 4 waves, 8 float4 loads in flight per lane (the whole 32 KiB chunk),
    // eight workgroups per CU: the fastest single-launch 64 MiB read measured
    // (tools/ubench_stream.hip; 8 waves with 4 loads, four per CU: no faster)
    const bool ef = a.resid != nullptr;
    constexpr uint32_t per_cu = 8u;
    const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(a.nc, per_cu * (uint32_t)num_cu));
    // the finish's roles: the last `fin` workgroups of the grid, at least
    // nwk + 1 of them (a ranker); else the fill launch finishes the call
    if (a.fin && (G < 2 * a.fin || a.fin <= a.nwk || a.nwk < 8 || a.nc > LMAXC || !a.tag)) a.fin = 0;
    if (a.gn) {  // the gather fused: fewer loads in flight per stream, more streams
        const uint32_t ns = (a.gres ? 1u : 0u) + a.gn - 1u;
        if (a.gn > GATHER_MAX) return hipErrorInvalidValue;
        if (ns <= 3) {
            if (ef) tv16_lscan<true, 4, 4, 3><<<G, 256, 0, s>>>(a);
            else tv16_lscan<false, 4, 4, 3><<<G, 256, 0, s>>>(a);
        } else if (ns <= 8) {
            if (ef) tv16_lscan<true, 4, 2, 8><<<G, 256, 0, s>>>(a);
            else tv16_lscan<false, 4, 2, 8><<<G, 256, 0, s>>>(a);
        } else {
            if (ef) tv16_lscan<true, 4, 1, GATHER_MAX><<<G, 256, 0, s>>>(a);
            else tv16_lscan<false, 4, 1, GATHER_MAX><<<G, 256, 0, s>>>(a);
        }
    } else {
        if (ef) tv16_lscan<true, 4, 8, 0><<<G, 256, 0, s>>>(a);
        else tv16_lscan<false, 4, 8, 0><<<G, 256, 0, s>>>(a);
    }
    return hipGetLastError();
}

}  // namespace stg
