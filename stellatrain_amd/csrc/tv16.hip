// tv16.hip -- thresholdv16 ("cache-aware" threshold-v) on gfx950.
//
// Reference: ThresholdvCompressor16::impl_simd_v2
// (/root/reference/backend/src/compress/thresholdv16.cpp:78-295), first
// threshold impl_get_first_threshold (:36-54), block sum hsum_float_avx (:57-73).
//
// Semantics: walk 16-float lines in index order; a line whose
// tree-ordered |x| sum S >= t is emitted whole while >= 16 slots remain
// (stage 1); with r = dst_len % 16 slots left the next qualifying line donates
// its first r elements (stage 2); a ragged tail is judged on its *signed* sum
// (stage 3); if the scan ran dry the rest is filled from the non-qualifying
// lines in descending-sum order (heap fill).  AIMD: t *= 0.99 (in double) when
// the scan ran dry, t += inc otherwise.
//
// GPU structure (two launches per call, first calls add a radix select):
//   tv16_scan  streaming pass over the bucket: one tree sum per line (a quad of
//              lanes per line, DPP cross-lane adds in the AVX order), sums to
//              scratch, per-tile qualifier counts.  HBM-bound: 4n bytes read.
//   tv16_fill  persistent, one workgroup per CU: global prefix of tile counts,
//              ordered emission of the first kb(+1) qualifying lines (gathered
//              from src), stage-3 tail, device-side AIMD update; in regime B a
//              radix descent over the sums (relative bins just below t, one grid
//              barrier per level), candidate collection and a last-arriver LDS
//              sort that orders the heap fill by (sum desc, position asc).
#include <algorithm>

#include "ws.h"

namespace stg {

namespace {

constexpr uint32_t L1_SHIFT = 14;  // level-1 bin width in ulps below t (~0.2% of t)

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
// scan: tree sums (AVX order), scratch sums, per-tile qualifier counts
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(STG_WG) tv16_scan(const float *__restrict__ src, uint32_t nb,
                                                    const KeyState *__restrict__ state, CallParams *cp,
                                                    float *__restrict__ sums, uint32_t *__restrict__ tile_cnt,
                                                    FillCtl *ctl, uint32_t nwg_fill) {
    const float t = state->t;
    if (blockIdx.x == 0) {
        // reset the fill kernel's control block for this call
        uint32_t *z = reinterpret_cast<uint32_t *>(ctl);
        const uint32_t words = (uint32_t)(offsetof(FillCtl, wg_ties) / 4) + nwg_fill;
        for (uint32_t i = threadIdx.x; i < words; i += STG_WG) z[i] = 0;
        if (threadIdx.x == 0) { cp->t = t; cp->inc = state->inc; }
    }
    const uint32_t lane = __lane_id();
    const uint32_t wave = threadIdx.x >> 6;
    const uint32_t q = lane & 3;
    const uint32_t tile0 = blockIdx.x * TV16_TILE_BLOCKS;

    float4 v[TV16_UNROLL];
#pragma unroll
    for (uint32_t u = 0; u < TV16_UNROLL; ++u) {
        const uint32_t blk = tile0 + u * (STG_WG / 4) + wave * 16 + (lane >> 2);
        if (blk < nb) v[u] = *reinterpret_cast<const float4 *>(src + (size_t)blk * 16 + q * 4);
        else v[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t u = 0; u < TV16_UNROLL; ++u) {
        const uint32_t blk = tile0 + u * (STG_WG / 4) + wave * 16 + (lane >> 2);
        const float ax = fabsf(v[u].x), ay = fabsf(v[u].y), az = fabsf(v[u].z), aw = fabsf(v[u].w);
        // lanes (0,1) hold floats 0..7 of the line, lanes (2,3) floats 8..15:
        // p = |x_i| + |x_{i+4}| per half, h = (p0+p1)+(p2+p3), S = h_lo + h_hi
        const float px = ax + dpp_f<QP_XOR1>(ax);
        const float py = ay + dpp_f<QP_XOR1>(ay);
        const float pz = az + dpp_f<QP_XOR1>(az);
        const float pw = aw + dpp_f<QP_XOR1>(aw);
        const float h = (px + py) + (pz + pw);
        const float S = h + dpp_f<QP_XOR2>(h);
        const bool valid = blk < nb;
        if (valid && q == 0) sums[blk] = S;
        const bool flag = valid && q == 0 && S >= t;
        cnt += (uint32_t)__popcll(__ballot(flag));
    }
    __shared__ uint32_t s_cnt[STG_WAVES];
    if (lane == 0) s_cnt[wave] = cnt;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t c = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) c += s_cnt[w];
        tile_cnt[blockIdx.x] = c;
    }
}

// ---------------------------------------------------------------------------
// fill
// ---------------------------------------------------------------------------
struct FillArgs {
    const float *src;
    uint64_t n;
    uint32_t nb, tl, dst_len, kb, r, ntiles;
    int32_t idx_offset;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    const CallParams *cp;
    const float *sums;
    const uint32_t *tile_cnt;
    FillCtl *ctl;
    uint64_t *cand;
    uint32_t *fail;
};

template <bool VEC>
__device__ __forceinline__ void emit_line(const FillArgs &a, uint32_t pos, uint32_t off, uint32_t len) {
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

template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tv16_fill(FillArgs a) {
    __shared__ uint32_t s_hist[HBINS];
    __shared__ uint64_t s_sort[SORT_CAP];
    __shared__ uint32_t sh[STG_WAVES + 1];
    __shared__ uint64_t sh64[STG_WAVES];
    __shared__ uint32_t s_dec[8];

    const uint32_t G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
    const float t = a.cp->t;
    const float inc = a.cp->inc;
    const uint32_t tb = f2u(t);
    const uint32_t t_begin = (uint32_t)((uint64_t)w * a.ntiles / G);
    const uint32_t t_end = (uint32_t)((uint64_t)(w + 1) * a.ntiles / G);

    // ---- phase A: total qualifiers and this workgroup's starting rank ----
    uint64_t tot = 0, bef = 0;
    for (uint32_t i = tid; i < a.ntiles; i += STG_WG) {
        const uint32_t c = a.tile_cnt[i];
        tot += c;
        if (i < t_begin) bef += c;
    }
    const uint32_t Qtot = (uint32_t)wg_sum64(tot, sh64);
    uint32_t P = (uint32_t)wg_sum64(bef, sh64);

    // ---- regime (identical in every workgroup) ----
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

    // ---- phase B: ordered emission of qualifying lines (+ level-1 histogram) ----
    const uint32_t hi0 = tb - 1u;  // largest candidate key (keys u < tb)
    if (regimeB) {
        for (uint32_t i = tid; i < HBINS; i += STG_WG) s_hist[i] = 0;
        __syncthreads();
    }
    constexpr uint32_t PF = 8;  // tiles of sums prefetched per chunk (one latency per chunk)
    for (uint32_t c0t = t_begin; c0t < t_end; c0t += PF) {
        if (!regimeB && P >= lim) break;  // uniform: later tiles emit nothing
        float2 pre[PF];
#pragma unroll
        for (uint32_t j = 0; j < PF; ++j) {
            const uint32_t b0 = (c0t + j) * TV16_TILE_BLOCKS + 2 * tid;
            pre[j] = make_float2(0.f, 0.f);
            if (c0t + j < t_end) {
                if (b0 + 1 < a.nb) pre[j] = *reinterpret_cast<const float2 *>(a.sums + b0);
                else if (b0 < a.nb) pre[j].x = a.sums[b0];
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < PF; ++j) {
            const uint32_t tile = c0t + j;
            if (tile >= t_end || (!regimeB && P >= lim)) break;
            const uint32_t b0 = tile * TV16_TILE_BLOCKS + 2 * tid;
            const float s0 = pre[j].x, s1 = pre[j].y;
            const bool v0 = b0 < a.nb, v1 = b0 + 1 < a.nb;
            const bool f0 = v0 && s0 >= t, f1 = v1 && s1 >= t;
            uint32_t tcount;
            const uint32_t ex = wg_excl_scan((uint32_t)f0 + (uint32_t)f1, sh, &tcount);
            const uint32_t g0 = P + ex, g1 = g0 + (uint32_t)f0;
            if (f0 && g0 < lim) emit_line<VEC>(a, b0 * 16, 16 * g0, g0 == a.kb ? a.r : 16u);
            if (f1 && g1 < lim) emit_line<VEC>(a, (b0 + 1) * 16, 16 * g1, g1 == a.kb ? a.r : 16u);
            if (regimeB) {
                const uint32_t u0 = f2u(s0), u1 = f2u(s1);
                if (v0 && !f0 && u0 < tb) atomicAdd(&s_hist[std::min((hi0 - u0) >> L1_SHIFT, HBINS - 1)], 1u);
                if (v1 && !f1 && u1 < tb) atomicAdd(&s_hist[std::min((hi0 - u1) >> L1_SHIFT, HBINS - 1)], 1u);
            }
            P += tcount;
        }
    }

    // ---- phase C: tail, AIMD, count ----
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

    // ---- phase D: heap fill = top candidates by (sum desc, position asc) ----
    const uint32_t rem = a.dst_len - cnt;
    const uint32_t nc = a.nb - Qtot;  // non-qualifying full lines
    const uint32_t M = std::min((rem + 15u) / 16u, nc);
    uint32_t nbar = 0;
    FillCtl *ctl = a.ctl;

    __syncthreads();
    for (uint32_t i = tid; i < HBINS; i += STG_WG)
        if (s_hist[i]) atomicAdd(&ctl->hist[0][i], s_hist[i]);

    // mode 1: collect keys >= blo and sort; mode 2: ties at ustar
    uint32_t mode = 1, blo = tb, ustar = 0, greater = 0, need_eq = 0;
    if (M > 0) {
        grid_barrier(&ctl->bar, ++nbar * G, a.fail);
        uint32_t lvl = 0, hi = hi0, lo = 0, s = L1_SHIFT, above = 0;
        bool ovf = true;
        for (;;) {
            // locate the bin holding rank `need` (1-based) counting down from hi
            const uint32_t need = M - above;
            uint32_t c[HBINS / STG_WG], sum = 0;
#pragma unroll
            for (uint32_t j = 0; j < HBINS / STG_WG; ++j) {
                c[j] = ld_acq_relaxed(&ctl->hist[lvl][tid * (HBINS / STG_WG) + j]);
                sum += c[j];
            }
            uint32_t total;
            const uint32_t before = wg_excl_scan(sum, sh, &total);
            if (tid == 0) { s_dec[0] = 0xffffffffu; s_dec[1] = 0; s_dec[2] = 0; }
            __syncthreads();
            if (need > before && need <= before + sum) {
                uint32_t acc = before;
                for (uint32_t j = 0; j < HBINS / STG_WG; ++j) {
                    if (need <= acc + c[j]) { s_dec[0] = tid * (HBINS / STG_WG) + j; s_dec[1] = acc; s_dec[2] = c[j]; break; }
                    acc += c[j];
                }
            }
            __syncthreads();
            const uint32_t bstar = s_dec[0], cum = s_dec[1], hb = s_dec[2];
            __syncthreads();
            if (bstar == 0xffffffffu) {  // histogram does not reach `need`: collect all
                if (tid == 0) atomicOr(a.fail, (uint32_t)FAIL_LEVELS);
                mode = 1; blo = 0;
                break;
            }
            if (ovf && bstar == HBINS - 1) {
                above += cum;
                const uint64_t width = (uint64_t)(HBINS - 1) << s;
                if ((uint64_t)hi < width) {  // cannot happen: bin would be empty
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
                if (s == 0) { mode = 2; ustar = bhi; greater = above + cum; need_eq = need - cum; break; }
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
            // histogram of this workgroup's candidates inside [lo, hi]
            for (uint32_t i = tid; i < HBINS; i += STG_WG) s_hist[i] = 0;
            __syncthreads();
            const uint32_t b_begin = t_begin * TV16_TILE_BLOCKS;
            const uint32_t b_end = std::min(t_end * TV16_TILE_BLOCKS, a.nb);
            for (uint32_t b = b_begin + tid; b < b_end; b += STG_WG) {
                const uint32_t u = f2u(a.sums[b]);
                if (u < tb && u >= lo && u <= hi) atomicAdd(&s_hist[(hi - u) >> s], 1u);
            }
            __syncthreads();
            for (uint32_t i = tid; i < HBINS; i += STG_WG)
                if (s_hist[i]) atomicAdd(&ctl->hist[lvl][i], s_hist[i]);
            grid_barrier(&ctl->bar, ++nbar * G, a.fail);
        }
    }

    const uint32_t b_begin = t_begin * TV16_TILE_BLOCKS;
    const uint32_t b_end = std::min(t_end * TV16_TILE_BLOCKS, a.nb);
    const uint32_t tailpos = a.nb * 16;
    const bool tail_in_greater = tail_cand && mode == 2 && tail_key > u2f(ustar);
    // collect: mode 1 -> keys in [blo, tb); mode 2 -> keys in (ustar, tb)
    if (M > 0) {
        const uint32_t kmin = mode == 1 ? blo : ustar + 1;
        for (uint32_t b0 = b_begin; b0 < b_end; b0 += STG_WG) {
            const uint32_t b = b0 + tid;
            uint32_t u = 0;
            bool p = false;
            if (b < b_end) { u = f2u(a.sums[b]); p = u < tb && u >= kmin; }
            const uint32_t slot = wave_append(&ctl->cand_n, p);
            if (p && slot < SORT_CAP)
                a.cand[slot] = ((uint64_t)(~(u | 0x80000000u)) << 32) | (uint64_t)(b * 16);
        }
    }
    if (mode == 2) {
        // ties at ustar, taken in position order: per-workgroup counts first
        uint32_t mine = 0;
        for (uint32_t b = b_begin + tid; b < b_end; b += STG_WG) mine += f2u(a.sums[b]) == ustar;
        const uint32_t my_ties = (uint32_t)wg_sum64(mine, sh64);
        if (tid == 0) ctl->wg_ties[w] = my_ties;
    }
    grid_barrier(&ctl->bar, ++nbar * G, a.fail);  // every append / tie count is visible
    if (mode == 2) {
        uint64_t pb = 0, pt = 0;
        for (uint32_t i = tid; i < G; i += STG_WG) {
            const uint32_t x = ld_acq_relaxed(&ctl->wg_ties[i]);
            pt += x;
            if (i < w) pb += x;
        }
        uint32_t rank = (uint32_t)wg_sum64(pb, sh64);
        const uint32_t all_ties = (uint32_t)wg_sum64(pt, sh64);
        const uint32_t base = cnt + 16u * greater + (tail_in_greater ? a.tl : 0u);
        for (uint32_t b0 = b_begin; b0 < b_end; b0 += STG_WG) {
            const uint32_t b = b0 + tid;
            const bool p = b < b_end && f2u(a.sums[b]) == ustar;
            uint32_t n_here;
            const uint32_t ex = wg_excl_scan((uint32_t)p, sh, &n_here);
            if (p) {
                const uint64_t off = (uint64_t)base + 16ull * (rank + ex);
                if (off < a.dst_len)
                    emit_line<VEC>(a, b * 16, (uint32_t)off, std::min<uint32_t>(16u, a.dst_len - (uint32_t)off));
            }
            rank += n_here;
        }
        if (w == 0 && tid == 0 && tail_cand && tail_key == u2f(ustar)) {
            const uint64_t off = (uint64_t)base + 16ull * all_ties;
            if (off < a.dst_len)
                emit_line<false>(a, tailpos, (uint32_t)off, std::min<uint32_t>(a.tl, a.dst_len - (uint32_t)off));
        }
        (void)need_eq;
    }

    // ---- distributed rank-and-emit of the collected set ----
    // Output order is (sum desc, position asc) = ascending composite key
    // (~ord(sum) << 32 | pos); an entry's rank is the number of smaller keys,
    // counted by one wave per entry over the LDS copy of the set.
    uint32_t nc_all = ld_acq_relaxed(&ctl->cand_n);
    if (nc_all > SORT_CAP) {
        if (w == 0 && tid == 0) atomicOr(a.fail, (uint32_t)FAIL_CAND_OVERFLOW);
        nc_all = SORT_CAP;
    }
    const bool add_tail = tail_cand && (mode == 1 || tail_in_greater) && nc_all < SORT_CAP;
    const uint32_t total = nc_all + (add_tail ? 1u : 0u);
    if (w >= total) return;
    const uint64_t tail_comp = ((uint64_t)(~ford(tail_key)) << 32) | (uint64_t)tailpos;
    for (uint32_t i = tid; i < total; i += STG_WG) s_sort[i] = i < nc_all ? a.cand[i] : tail_comp;
    __syncthreads();
    const uint32_t lane = __lane_id(), wv = tid >> 6;
    for (uint32_t e = w + G * wv; e < total; e += G * STG_WAVES) {
        const uint64_t key = s_sort[e];
        uint32_t less = 0;
        for (uint32_t j = lane; j < total; j += 64) less += s_sort[j] < key;
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
}

}  // namespace

hipError_t launch_tv16(const Tv16Launch &a, const DevWS &ws, hipStream_t s) {
    const uint32_t nb = (uint32_t)(a.n / 16);
    const uint32_t tl = (uint32_t)(a.n % 16);
    const uint32_t ntiles = (nb + TV16_TILE_BLOCKS - 1) / TV16_TILE_BLOCKS;
    if (a.first) {
        const uint32_t nblk = (uint32_t)((a.n + 15) / 16);
        tv16_seq_sums<<<(nblk + STG_WG - 1) / STG_WG, STG_WG, 0, s>>>(a.src, a.n, ws.sums, nblk);
        const uint32_t bk = std::min<uint32_t>(a.k / 16, nblk - 1);
        hipError_t e = launch_radix_select(ws.sums, nblk, 0xffffffffu, 0, nullptr, bk, ws, a.num_cu, s);
        if (e != hipSuccess) return e;
        tv16_init_state<<<1, 1, 0, s>>>(a.state, ws.rsel);
    }
    const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>(std::min<uint32_t>((uint32_t)a.num_cu, ntiles), MAX_FILL_WG));
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    tv16_scan<<<std::max<uint32_t>(1, ntiles), STG_WG, 0, s>>>(a.src, nb, a.state, ws.cp, ws.sums, ws.tile_cnt,
                                                             ws.ctl, G);
    FillArgs f;
    f.src = a.src;
    f.n = a.n;
    f.nb = nb;
    f.tl = tl;
    f.dst_len = a.dst_len;
    f.kb = a.dst_len / 16;
    f.r = a.dst_len % 16;
    f.ntiles = ntiles;
    f.idx_offset = a.idx_offset;
    f.idx = a.idx;
    f.val = a.val;
    f.count_out = a.count_out;
    f.state = a.state;
    f.cp = ws.cp;
    f.sums = ws.sums;
    f.tile_cnt = ws.tile_cnt;
    f.ctl = ws.ctl;
    f.cand = ws.cand;
    f.fail = ws.fail;
    const bool vec = ((reinterpret_cast<uintptr_t>(a.src) | reinterpret_cast<uintptr_t>(a.idx) |
                       reinterpret_cast<uintptr_t>(a.val)) & 15u) == 0;
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    if (vec) tv16_fill<true><<<G, STG_WG, 0, s>>>(f);
    else tv16_fill<false><<<G, STG_WG, 0, s>>>(f);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}

}  // namespace stg
