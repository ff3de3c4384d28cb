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
// One persistent launch per call (tv16_fused), one workgroup per CU, each
// owning a contiguous range of lines:
//   1. stream its range once (quad of lanes per line, DPP cross-lane adds in
//      the AVX tree order), keep the line sums in LDS, count S >= t;
//   2. publish the count as an epoch-tagged 8-byte granule and gather all
//      granules (no memset per call, no acquire needed: only atomics cross);
//   3. every workgroup derives the same regime; emit its qualifying lines
//      with global rank < kb (+1 partial) straight from src (L2/MALL hot);
//   4. workgroup 0 writes the stage-3 tail, the AIMD threshold and the count;
//   5. regime B only: radix descent over the LDS sums (relative bins just
//      below t, one grid barrier per level), candidate collection, and a
//      distributed rank-and-emit that orders the heap fill by
//      (sum desc, position asc).
// First calls run tv16_seq_sums + radix select (select.hip) before it.
#include <algorithm>
#include <cstdlib>

#include "ws.h"

namespace stg {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

constexpr uint32_t FWG = 1024;        // fused-kernel workgroup: 16 waves, two per CU
constexpr uint32_t FNW = FWG / 64;
constexpr uint32_t L1_SHIFT = 14;     // level-1 bin width in ulps below t (~0.2% of t)
constexpr uint32_t LDS_LINES = SORT_CAP * 2;  // line sums cached in LDS per workgroup
constexpr uint32_t SCAN_U = 8;        // float4 per lane per batch (two batches in flight)
constexpr uint32_t MAX_J = LDS_LINES / FWG;
constexpr uint32_t WIN = 1u << 17;    // regime-B window below t, in ulps (~1.6% of t)
constexpr uint32_t STAGE_LINES = 256;  // qualifying lines staged in LDS per workgroup (16 KiB)

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

struct FusedArgs {
    const float *src;
    uint64_t n;
    uint32_t nb, tl, dst_len, kb, r, epoch;
    int32_t idx_offset;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    float *sums_g;  // global line sums when a range exceeds LDS_LINES
    FillCtl *ctl;
    uint64_t *cand;
    uint32_t *fail;
};

template <bool VEC>
__device__ __forceinline__ void emit_line(const FusedArgs &a, uint32_t pos, uint32_t off, uint32_t len) {
    if (VEC && len == 16) {
        const float4 *s4 = reinterpret_cast<const float4 *>(a.src + pos);
        float4 *v4 = reinterpret_cast<float4 *>(a.val + off);
        uint4 *i4 = reinterpret_cast<uint4 *>(a.idx + off);
        const uint32_t b = pos + (uint32_t)a.idx_offset;
        const float4 x0 = s4[0], x1 = s4[1], x2 = s4[2], x3 = s4[3];
        v4[0] = x0; v4[1] = x1; v4[2] = x2; v4[3] = x3;
        i4[0] = make_uint4(b + 0, b + 1, b + 2, b + 3);
        i4[1] = make_uint4(b + 4, b + 5, b + 6, b + 7);
        i4[2] = make_uint4(b + 8, b + 9, b + 10, b + 11);
        i4[3] = make_uint4(b + 12, b + 13, b + 14, b + 15);
    } else {
        for (uint32_t i = 0; i < len; ++i) {
            a.val[off + i] = a.src[(size_t)pos + i];
            a.idx[off + i] = pos + i + (uint32_t)a.idx_offset;
        }
    }
}

__device__ __forceinline__ uint32_t bitlen(uint32_t x) { return x ? 32u - __clz(x) : 0u; }

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

// STAGE (diagnostics only, STG_DEBUG_TV16_STAGE): 0 = full codec; 1 = return
// after the streaming pass; 2 = after the count exchange; 3 = plain streaming
// read (calibration); 4 = full codec + per-workgroup phase stamps.
template <bool VEC, bool LDS_SUMS, int STAGE = 0>
__global__ void __launch_bounds__(FWG, 8) tv16_fused(FusedArgs a) {
    __shared__ uint64_t s_buf[SORT_CAP];  // line sums (floats) in 1-5, candidates at the end
    __shared__ float4 s_stage[STAGE_LINES * 4];  // qualifying lines, staged during the scan
    __shared__ uint32_t s_stage_line[STAGE_LINES];
    __shared__ uint64_t s_mask[MAX_J * FNW];
    __shared__ uint32_t s_hist[HBINS];
    __shared__ uint32_t s_wt[MAX_J * FNW + 1];
    __shared__ uint32_t sh[FNW + 1];
    __shared__ uint64_t sh64[FNW];
    __shared__ uint32_t s_dec[8];
    __shared__ uint32_t s_nst;
    float *s_sum = reinterpret_cast<float *>(s_buf);
#define STAMP(k_)                                                                                   \
    do {                                                                                            \
        if (STAGE == 4 && threadIdx.x == 0)                                                         \
            a.count_out[1 + blockIdx.x * 16 + (k_)] = (uint32_t)__builtin_amdgcn_s_memrealtime(); \
    } while (0)

    const uint32_t G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
    const uint32_t lane = __lane_id(), wave = tid >> 6, q = lane & 3;
    const uint32_t L0 = (uint32_t)((uint64_t)w * a.nb / G);
    const uint32_t L1 = (uint32_t)((uint64_t)(w + 1) * a.nb / G);
    const uint32_t nl = L1 - L0;
    FillCtl *ctl = a.ctl;
    CallCtl *cc = &ctl->cc[a.epoch & 1u];
    const uint64_t tag = (uint64_t)a.epoch << 32;
    // Every workgroup reads the state before it arrives at the count exchange;
    // workgroup 0 rewrites the state only after the exchange completed.
    const float t = a.state->t;
    const float inc = a.state->inc;
    const uint32_t tb = f2u(t);
    const uint32_t wlo = tb > WIN ? tb - WIN : 0u;  // window [wlo, tb) just below t

    auto put_sum = [&](uint32_t i, float S) {
        if (LDS_SUMS) s_sum[i] = S;
        else a.sums_g[L0 + i] = S;
    };
    auto get_sum = [&](uint32_t i) -> float { return LDS_SUMS ? s_sum[i] : a.sums_g[L0 + i]; };
    // Last-arriver grid barrier, round r (1-based): the workgroup whose arrival
    // completes the round writes every workgroup's own go word.
    auto grid_sync = [&](uint32_t r) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) s_dec[7] = __hip_atomic_fetch_add(&cc->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (s_dec[7] == r * G - 1) {
            if (tid < G) st_sc1(&ctl->slot[tid].go, tag | r);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (tid == 0) {
            for (uint32_t spins = 0; ld_sc1(&ctl->slot[w].go) != (tag | r); ++spins) {
                __builtin_amdgcn_s_sleep(1);
                if (spins > (1u << 24)) { atomicOr(a.fail, (uint32_t)FAIL_SPIN_TIMEOUT); break; }
            }
        }
        __syncthreads();
    };

    if (tid == 0) s_nst = 0;
    __syncthreads();
    STAMP(0);
    if (STAGE == 4 && tid == 0) a.count_out[1 + w * 16 + 8] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));

    // ---- 1. stream the range: line sums, qualifier count (+ staging), window count ----
    uint32_t cnt_w = 0, win_w = 0;
    {
        const uint32_t lane_line = wave * 16 + (lane >> 2);  // line of this lane in a step
        constexpr uint32_t STEP = FWG / 4;                   // lines per step
        const uint32_t nsteps = (nl + STEP - 1) / STEP;
        const uint32_t nbatch = (nsteps + SCAN_U - 1) / SCAN_U;
        const uint32_t leader = lane & ~3u;
        const uint64_t below_leader = leader ? (~0ull >> (64 - leader)) : 0ull;
        // One batch of SCAN_U float4 per lane in flight; the 32 waves per CU
        // (2 workgroups x 16 waves) supply the memory-level parallelism
        // (tools/ubench_stream.hip: 1 x 1024 threads/CU streams at ~4.0 TB/s,
        // 2 x 1024 at ~5.4-5.8, nontemporal loads +5%).  Loads are
        // straight-line: lanes past the range re-read line 0 of the range.
        for (uint32_t b = 0; b < nbatch; ++b) {
            float4 v[SCAN_U];
#pragma unroll
            for (uint32_t u = 0; u < SCAN_U; ++u) {
                const uint32_t i = (b * SCAN_U + u) * STEP + lane_line;
                const uint32_t ic = i < nl ? i : 0u;
                const f4v t4 = __builtin_nontemporal_load(
                    reinterpret_cast<const f4v *>(a.src + (size_t)(L0 + ic) * 16 + q * 4));
                v[u] = make_float4(t4.x, t4.y, t4.z, t4.w);
            }
#pragma unroll
            for (uint32_t u = 0; u < SCAN_U; ++u) {
                const uint32_t i = (b * SCAN_U + u) * STEP + lane_line;
                if (STAGE == 3) {
                    cnt_w += f2u(v[u].x + v[u].y + v[u].z + v[u].w) == 0x7f800001u;
                    continue;
                }
                const float S = quad_line_sum(v[u]);
                const bool lead = i < nl && q == 0;
                if (lead) put_sum(i, S);
                const uint32_t us = f2u(S);
                const uint64_t bq = __ballot(lead && S >= t);
                win_w += (uint32_t)__popcll(__ballot(lead && us >= wlo && us < tb));
                if (bq) {  // stage the qualifying lines (all four lanes of each quad)
                    cnt_w += (uint32_t)__popcll(bq);
                    uint32_t base = 0;
                    if (lane == 0) base = atomicAdd(&s_nst, (uint32_t)__popcll(bq));
                    base = __shfl(base, 0, 64);
                    if ((bq >> leader) & 1ull) {
                        const uint32_t slot = base + (uint32_t)__popcll(bq & below_leader);
                        if (slot < STAGE_LINES) {
                            s_stage[slot * 4 + q] = v[u];
                            if (q == 0) s_stage_line[slot] = i;
                        }
                    }
                }
            }
        }
    }
    if (STAGE == 1 || STAGE == 3) {
        if (cnt_w == 12345u) a.count_out[1] = win_w;  // keep the loop alive
        return;
    }
    if (lane == 0) { s_wt[wave] = cnt_w; s_wt[FNW + wave] = win_w; }
    __syncthreads();
    uint32_t Qw = 0, Ww = 0;
#pragma unroll
    for (uint32_t i = 0; i < FNW; ++i) { Qw += s_wt[i]; Ww += s_wt[FNW + i]; }
    __syncthreads();

    STAMP(1);
    // ---- 2. count exchange: publish {epoch | count} and {epoch | window count},
    //         then one wave gathers every workgroup's granules: all slots'
    //         loads in flight at once, re-polling only the stale ones ----
    if (tid == 0) {
        st_sc1(&ctl->gran[w], tag | Qw);
        st_sc1(&ctl->gran2[w], tag | Ww);
    }
    if (wave == 0) {
        constexpr uint32_t SL = MAX_FILL_WG / 64;
        uint64_t g[SL], g2[SL];
        uint32_t pending = 0;
#pragma unroll
        for (uint32_t j = 0; j < SL; ++j) {
            g[j] = g2[j] = 0;
            if (j * 64 + lane < G) pending |= 1u << j;
        }
        for (uint32_t spins = 0;; ++spins) {
#pragma unroll
            for (uint32_t j = 0; j < SL; ++j)
                if ((pending >> j) & 1u) {
                    g[j] = ld_sc1(&ctl->gran[j * 64 + lane]);
                    g2[j] = ld_sc1(&ctl->gran2[j * 64 + lane]);
                }
#pragma unroll
            for (uint32_t j = 0; j < SL; ++j)
                if (((pending >> j) & 1u) && (g[j] >> 32) == a.epoch && (g2[j] >> 32) == a.epoch)
                    pending &= ~(1u << j);
            if (!__any(pending != 0)) break;
            __builtin_amdgcn_s_sleep(2);
            if (spins > (1u << 22)) { atomicOr(a.fail, (uint32_t)FAIL_SPIN_TIMEOUT); break; }
        }
        uint64_t bef = 0, tot = 0, wbef = 0, wtot = 0;
#pragma unroll
        for (uint32_t j = 0; j < SL; ++j) {
            const uint32_t vv = j * 64 + lane;
            if (vv < G) {
                const uint64_t c = (uint32_t)g[j], cw = (uint32_t)g2[j];
                tot += c;
                wtot += cw;
                if (vv < w) { bef += c; wbef += cw; }
            }
        }
        bef = wave_sum64(bef);
        tot = wave_sum64(tot);
        wbef = wave_sum64(wbef);
        wtot = wave_sum64(wtot);
        if (lane == 0) {
            s_dec[0] = (uint32_t)bef;
            s_dec[1] = (uint32_t)tot;
            s_dec[5] = (uint32_t)wtot;
            s_dec[6] = (uint32_t)wbef;
        }
    }
    __syncthreads();
    const uint32_t P = s_dec[0];
    const uint32_t Qtot = s_dec[1];
    const uint32_t Wtot = s_dec[5];
    const uint32_t Wbef = s_dec[6];
    if (STAGE == 2) return;

    STAMP(2);
    // ---- 3. regime (identical in every workgroup) ----
    const uint32_t lim = a.kb + (a.r ? 1u : 0u);
    const uint32_t c0 = Qtot >= lim ? a.dst_len : 16u * Qtot;
    bool tail_q = false, tail_cand = false;
    float tail_key = 0.f;
    uint32_t ct = 0;
    if (c0 < a.dst_len && a.tl) {
        const float *tp = a.src + (size_t)a.nb * 16;
        float s = 0.f;
        for (uint32_t i = 0; i < a.tl; ++i) s += tp[i];
        tail_q = s * 16.0f >= t * (float)a.tl;
        if (tail_q) ct = std::min(a.dst_len - c0, a.tl);
        else { tail_cand = true; tail_key = s * 16.0f / (float)a.tl; }
    }
    const uint32_t cnt = c0 + ct;
    const bool regimeB = cnt < a.dst_len;

    // ---- 3b. ordered emission of this range's qualifying lines ----
    // In-range rank of line i = j*FWG + tid via ballot masks (order j, wave, lane).
    if (P < lim && Qw) {
        const uint32_t nj = (nl + FWG - 1) / FWG;
        const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
        if (nj <= MAX_J && Qw <= STAGE_LINES) {
            // every qualifying line is staged in LDS: one thread per staged line
            for (uint32_t j = 0; j < nj; ++j) {
                const uint32_t i = j * FWG + tid;
                const uint64_t bal = __ballot(i < nl && get_sum(i) >= t);
                if (lane == 0) { s_mask[j * FNW + wave] = bal; s_wt[j * FNW + wave] = (uint32_t)__popcll(bal); }
            }
            __syncthreads();
            if (tid == 0) {
                uint32_t acc = 0;
                for (uint32_t i = 0; i < nj * FNW; ++i) { const uint32_t x = s_wt[i]; s_wt[i] = acc; acc += x; }
            }
            __syncthreads();
            for (uint32_t e = tid; e < Qw; e += FWG) {
                const uint32_t i = s_stage_line[e];
                const uint32_t grp = (i / FWG) * FNW + ((i % FWG) >> 6), ln = i & 63;
                const uint64_t m = s_mask[grp];
                const uint32_t g = P + s_wt[grp] + (uint32_t)__popcll(m & (ln ? (~0ull >> (64 - ln)) : 0ull));
                if (g < lim) {
                    const uint32_t pos = (L0 + i) * 16;
                    const uint32_t len = g == a.kb ? a.r : 16u;
                    const uint32_t off = 16 * g;
                    if (VEC && len == 16) {
                        float4 *v4 = reinterpret_cast<float4 *>(a.val + off);
                        uint4 *i4 = reinterpret_cast<uint4 *>(a.idx + off);
                        const uint32_t bi = pos + (uint32_t)a.idx_offset;
#pragma unroll
                        for (uint32_t c = 0; c < 4; ++c) {
                            v4[c] = s_stage[e * 4 + c];
                            i4[c] = make_uint4(bi + 4 * c, bi + 4 * c + 1, bi + 4 * c + 2, bi + 4 * c + 3);
                        }
                    } else {
                        const float *sv = reinterpret_cast<const float *>(&s_stage[e * 4]);
                        for (uint32_t c = 0; c < len; ++c) {
                            a.val[off + c] = sv[c];
                            a.idx[off + c] = pos + c + (uint32_t)a.idx_offset;
                        }
                    }
                }
            }
        } else {
            // staging overflowed (low threshold): re-read the lines from src
            uint32_t base = P;
            for (uint32_t j0 = 0; j0 < nj && base < lim; j0 += MAX_J) {
                const uint32_t jn = std::min(nj - j0, MAX_J);
                uint32_t flags = 0;
                for (uint32_t j = 0; j < jn; ++j) {
                    const uint32_t i = (j0 + j) * FWG + tid;
                    const bool f = i < nl && get_sum(i) >= t;
                    flags |= (uint32_t)f << j;
                    const uint64_t bal = __ballot(f);
                    if (lane == 0) s_wt[j * FNW + wave] = (uint32_t)__popcll(bal);
                }
                __syncthreads();
                if (tid == 0) {
                    uint32_t acc = 0;
                    for (uint32_t i = 0; i < jn * FNW; ++i) { const uint32_t x = s_wt[i]; s_wt[i] = acc; acc += x; }
                    s_wt[MAX_J * FNW] = acc;
                }
                __syncthreads();
                for (uint32_t j = 0; j < jn; ++j) {
                    const uint64_t bal = __ballot((flags >> j) & 1u);
                    if ((flags >> j) & 1u) {
                        const uint32_t g = base + s_wt[j * FNW + wave] + (uint32_t)__popcll(bal & lt);
                        if (g < lim) {
                            const uint32_t line = L0 + (j0 + j) * FWG + tid;
                            emit_line<VEC>(a, line * 16, 16 * g, g == a.kb ? a.r : 16u);
                        }
                    }
                }
                base += s_wt[MAX_J * FNW];
                __syncthreads();
            }
        }
    }

    STAMP(3);
    // ---- 4. tail, AIMD, count (workgroup 0) ----
    if (w == 0) {  // zero the next call's counters (this call never touches them)
        uint32_t *z = reinterpret_cast<uint32_t *>(&ctl->cc[(a.epoch + 1) & 1u]);
        for (uint32_t i = tid; i < sizeof(CallCtl) / 4; i += FWG) st_sc1(z + i, 0u);
    }
    if (w == 0 && tid == 0) {
        if (ct) {
            const size_t p0 = (size_t)a.nb * 16;
            for (uint32_t i = 0; i < ct; ++i) {
                a.val[c0 + i] = a.src[p0 + i];
                a.idx[c0 + i] = (uint32_t)(p0 + i) + (uint32_t)a.idx_offset;
            }
        }
        a.state->t = regimeB ? (float)((double)t * 0.99) : t + inc;
        a.state->inc = inc;
        a.state->init = 1;
        *a.count_out = (uint32_t)std::min<uint64_t>(a.dst_len, a.n);
    }
    if (!regimeB) return;

    // ---- 5. heap fill = top candidates by (sum desc, position asc) ----
    const uint32_t rem = a.dst_len - cnt;
    const uint32_t nc = a.nb - Qtot;  // non-qualifying full lines
    const uint32_t M = std::min((rem + 15u) / 16u, nc);
    const uint32_t hi0 = tb - 1u;     // largest candidate key (keys u < tb)
    uint32_t nbar = 0;

    // mode 1: collect keys >= blo; mode 2: ties at ustar taken in position order
    uint32_t mode = 1, blo = tb, ustar = 0, greater = 0;
    if (M > 0 && Wtot >= M && Wtot + 1 <= SORT_CAP) {
        blo = wlo;  // the window holds the top M: no histogram needed
    } else if (M > 0) {
        for (uint32_t i = tid; i < HBINS; i += FWG) s_hist[i] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < nl; i += FWG) {
            const uint32_t u = f2u(get_sum(i));
            if (u < tb) atomicAdd(&s_hist[std::min((hi0 - u) >> L1_SHIFT, HBINS - 1)], 1u);
        }
        __syncthreads();
        for (uint32_t i = tid; i < HBINS; i += FWG)
            if (s_hist[i]) atomicAdd(&cc->hist[0][i], s_hist[i]);
        grid_sync(++nbar);
        uint32_t lvl = 0, hi = hi0, lo = 0, s = L1_SHIFT, above = 0;
        bool ovf = true;
        for (;;) {
            // locate the bin holding rank `need` (1-based) counting down from hi
            const uint32_t need = M - above;
            const uint32_t cbin = tid < HBINS ? ld_acq_relaxed(&cc->hist[lvl][tid]) : 0u;
            uint32_t total;
            const uint32_t before = blk_excl_scan<FNW>(cbin, sh, &total);
            if (tid == 0) { s_dec[2] = 0xffffffffu; s_dec[3] = 0; s_dec[4] = 0; }
            __syncthreads();
            if (tid < HBINS && need > before && need <= before + cbin) { s_dec[2] = tid; s_dec[3] = before; s_dec[4] = cbin; }
            __syncthreads();
            const uint32_t bstar = s_dec[2], cum = s_dec[3], hb = s_dec[4];
            __syncthreads();
            if (bstar == 0xffffffffu) {  // histogram does not reach `need`: collect all
                if (tid == 0) atomicOr(a.fail, (uint32_t)FAIL_LEVELS);
                mode = 1; blo = 0;
                break;
            }
            if (ovf && bstar == HBINS - 1) {
                above += cum;
                const uint64_t width = (uint64_t)(HBINS - 1) << s;
                if ((uint64_t)hi < width) {
                    if (tid == 0) atomicOr(a.fail, (uint32_t)FAIL_LEVELS);
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
                if (totc + 1 <= SORT_CAP) { mode = 1; blo = bl; break; }
                if (s == 0) { mode = 2; ustar = bhi; greater = above + cum; break; }
                above += cum;
                hi = bhi;
                lo = bl;
                s = s >= 10 ? s - 10 : 0;
            }
            if (++lvl >= MAX_LEVELS) {
                if (tid == 0) atomicOr(a.fail, (uint32_t)FAIL_LEVELS);
                mode = 1; blo = lo;
                break;
            }
            for (uint32_t i = tid; i < HBINS; i += FWG) s_hist[i] = 0;
            __syncthreads();
            for (uint32_t i = tid; i < nl; i += FWG) {
                const uint32_t u = f2u(get_sum(i));
                if (u < tb && u >= lo && u <= hi) atomicAdd(&s_hist[(hi - u) >> s], 1u);
            }
            __syncthreads();
            for (uint32_t i = tid; i < HBINS; i += FWG)
                if (s_hist[i]) atomicAdd(&cc->hist[lvl][i], s_hist[i]);
            grid_sync(++nbar);
        }
    }

    STAMP(4);
    const uint32_t tailpos = a.nb * 16;
    const bool tail_in_greater = tail_cand && mode == 2 && tail_key > u2f(ustar);
    // collect (write-through): mode 1 -> keys in [blo, tb); mode 2 -> keys in (ustar, tb).
    // The window path knows every workgroup's slot range from the exchanged
    // window counts (no atomics); the rare histogram paths append with one
    // atomic per workgroup and step.
    const bool win_path = mode == 1 && blo == wlo && M > 0 && Wtot >= M && Wtot + 1 <= SORT_CAP;
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
            const uint32_t ex = blk_excl_scan<FNW>((uint32_t)p, sh, &n_here);
            if (!n_here) continue;
            uint32_t base;
            if (win_path) {
                base = run;
                run += n_here;
            } else {
                if (tid == 0) s_dec[7] = atomicAdd(&cc->cand_n, n_here);
                __syncthreads();
                base = s_dec[7];
                __syncthreads();
            }
            if (p && base + ex < SORT_CAP)
                st_sc1(&a.cand[base + ex], ((uint64_t)(~(u | 0x80000000u)) << 32) | (uint64_t)((L0 + i) * 16));
        }
        if (mode == 2) {
            const uint32_t my_ties = (uint32_t)blk_sum64<FNW>(mine, sh64);
            if (tid == 0) st_sc1(&ctl->wg_ties[w], my_ties);
        }
    }
    STAMP(5);
    grid_sync(++nbar);  // every append / tie count is visible
    STAMP(6);
    if (mode == 2) {
        uint64_t pb = 0, pt = 0;
        for (uint32_t i = tid; i < G; i += FWG) {
            const uint32_t x = ld_acq_relaxed(&ctl->wg_ties[i]);
            pt += x;
            if (i < w) pb += x;
        }
        uint32_t rank = (uint32_t)blk_sum64<FNW>(pb, sh64);
        const uint32_t all_ties = (uint32_t)blk_sum64<FNW>(pt, sh64);
        const uint32_t base = cnt + 16u * greater + (tail_in_greater ? a.tl : 0u);
        for (uint32_t i0 = 0; i0 < nl; i0 += FWG) {
            const uint32_t i = i0 + tid;
            const bool p = i < nl && f2u(get_sum(i)) == ustar;
            uint32_t n_here;
            const uint32_t ex = blk_excl_scan<FNW>((uint32_t)p, sh, &n_here);
            if (p) {
                const uint64_t off = (uint64_t)base + 16ull * (rank + ex);
                if (off < a.dst_len)
                    emit_line<VEC>(a, (L0 + i) * 16, (uint32_t)off, std::min<uint32_t>(16u, a.dst_len - (uint32_t)off));
            }
            rank += n_here;
        }
        if (w == 0 && tid == 0 && tail_cand && tail_key == u2f(ustar)) {
            const uint64_t off = (uint64_t)base + 16ull * all_ties;
            if (off < a.dst_len)
                emit_line<false>(a, tailpos, (uint32_t)off, std::min<uint32_t>(a.tl, a.dst_len - (uint32_t)off));
        }
        __syncthreads();  // line sums in s_buf are dead from here on
    }

    // ---- distributed rank-and-emit of the collected set ----
    // Output order is (sum desc, position asc) = ascending composite key
    // (~ord(sum) << 32 | pos); an entry's rank is the number of smaller keys,
    // counted by one wave per entry over the LDS copy of the set.
    uint32_t nc_all = win_path ? Wtot : ld_acq_relaxed(&cc->cand_n);
    if (nc_all > SORT_CAP) {
        if (w == 0 && tid == 0) atomicOr(a.fail, (uint32_t)FAIL_CAND_OVERFLOW);
        nc_all = SORT_CAP;
    }
    const bool add_tail = tail_cand && (mode == 1 || tail_in_greater) && nc_all < SORT_CAP;
    const uint32_t total = nc_all + (add_tail ? 1u : 0u);
    const uint32_t first_e = w * FNW;  // entries handled here: e = w*FNW + wave + k*G*FNW
    if (first_e >= total) return;
    const uint64_t tail_comp = ((uint64_t)(~ford(tail_key)) << 32) | (uint64_t)tailpos;
    __syncthreads();
    for (uint32_t i = tid; i < total; i += FWG) s_buf[i] = i < nc_all ? ld_sc1(&a.cand[i]) : tail_comp;
    __syncthreads();
    for (uint32_t e = first_e + wave; e < total; e += G * FNW) {
        const uint64_t key = s_buf[e];
        uint32_t less = 0;
        for (uint32_t j = lane; j < total; j += 64) less += s_buf[j] < key;
        const uint32_t rank = wave_sum(less);
        const bool is_tail = add_tail && key == tail_comp;
        const bool tail_before = add_tail && tail_comp < key;
        const uint32_t pos = (uint32_t)key;
        const uint32_t len = is_tail ? a.tl : 16u;
        const uint64_t off = (uint64_t)cnt + 16ull * rank - (tail_before ? (uint64_t)(16u - a.tl) : 0ull);
        if (off < a.dst_len) {
            const uint32_t L = std::min<uint32_t>(len, a.dst_len - (uint32_t)off);
            if (lane < L) {
                a.val[off + lane] = a.src[(size_t)pos + lane];
                a.idx[off + lane] = pos + lane + (uint32_t)a.idx_offset;
            }
        }
    }
    STAMP(7);
#undef STAMP
}

}  // namespace

hipError_t launch_tv16(const Tv16Launch &a, const DevWS &ws, hipStream_t s) {
    const uint32_t nb = (uint32_t)(a.n / 16);
    const uint32_t tl = (uint32_t)(a.n % 16);
    if (a.first) {
        const uint32_t nblk = (uint32_t)((a.n + 15) / 16);
        tv16_seq_sums<<<(nblk + STG_WG - 1) / STG_WG, STG_WG, 0, s>>>(a.src, a.n, ws.sums, nblk);
        const uint32_t bk = std::min<uint32_t>(a.k / 16, nblk - 1);
        hipError_t e = launch_radix_select(ws.sums, nblk, 0xffffffffu, 0, nullptr, bk, ws, a.num_cu, s);
        if (e != hipSuccess) return e;
        tv16_init_state<<<1, 1, 0, s>>>(a.state, ws.rsel);
    }
    // wg_per_cu 1024-thread workgroups per CU (2: 32 waves, full occupancy for
    // one call; 1: half, so two calls from two streams share the CUs), all
    // co-resident for the in-launch exchanges, at least 1024 lines each
    const uint32_t G = std::max<uint32_t>(
        1, std::min<uint32_t>(std::min<uint32_t>(a.wg_per_cu * (uint32_t)a.num_cu, (nb + 1023) / 1024), MAX_FILL_WG));
    const uint32_t per = (nb + G - 1) / G;
    FusedArgs f;
    f.src = a.src;
    f.n = a.n;
    f.nb = nb;
    f.tl = tl;
    f.dst_len = a.dst_len;
    f.kb = a.dst_len / 16;
    f.r = a.dst_len % 16;
    f.epoch = a.epoch;
    f.idx_offset = a.idx_offset;
    f.idx = a.idx;
    f.val = a.val;
    f.count_out = a.count_out;
    f.state = a.state;
    f.sums_g = ws.sums;
    f.ctl = ws.ctl;
    f.cand = ws.cand;
    f.fail = ws.fail;
    const bool vec = ((reinterpret_cast<uintptr_t>(a.src) | reinterpret_cast<uintptr_t>(a.idx) |
                       reinterpret_cast<uintptr_t>(a.val)) & 15u) == 0;
    const bool lds = per <= LDS_LINES;
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    static const int dbg_stage = getenv("STG_DEBUG_TV16_STAGE") ? atoi(getenv("STG_DEBUG_TV16_STAGE")) : 0;
    if (dbg_stage == 1) tv16_fused<true, true, 1><<<G, FWG, 0, s>>>(f);
    else if (dbg_stage == 2) tv16_fused<true, true, 2><<<G, FWG, 0, s>>>(f);
    else if (dbg_stage == 3) tv16_fused<true, true, 3><<<G, FWG, 0, s>>>(f);
    else if (dbg_stage == 4) tv16_fused<true, true, 4><<<G, FWG, 0, s>>>(f);
    else if (vec && lds) tv16_fused<true, true><<<G, FWG, 0, s>>>(f);
    else if (vec) tv16_fused<true, false><<<G, FWG, 0, s>>>(f);
    else if (lds) tv16_fused<false, true><<<G, FWG, 0, s>>>(f);
    else tv16_fused<false, false><<<G, FWG, 0, s>>>(f);
    if (a.ev) {
        (void)hipEventRecord(a.ev[1], s);
        (void)hipEventRecord(a.ev[2], s);
    }
    return hipGetLastError();
}

}  // namespace stg
