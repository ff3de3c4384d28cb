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
// GPU structure: tv_scan streams the bucket (8192-element tiles, one float4
// per lane per step), stages each tile's qualifiers (in order) in a fixed
// per-tile slot and records per-tile counts and max|x|; tv_fill (one
// workgroup per CU) turns tile counts into global offsets, copies the staged
// pairs to their final place (re-deriving a tile from src in the rare case it
// overflowed its staging slot) and updates the threshold on the device.
#include <algorithm>

#include "tile.h"

namespace stg {

namespace {

__global__ void tv_init_state(KeyState *st, const RSel *rs) {
    st->t = u2f(rs->prefix);
    st->inc = 0.f;
    st->init = 1;
}

template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tv_scan(const float *__restrict__ src, size_t n,
                                                  const KeyState *__restrict__ state, uint32_t *__restrict__ tile_cnt,
                                                  uint32_t *__restrict__ tile_max, uint32_t *__restrict__ stage_pos,
                                                  float *__restrict__ stage_val, CallParams *cp) {
    __shared__ uint32_t s_wt[TILE_U * STG_WAVES + 1];
    __shared__ uint32_t s_max[STG_WAVES];
    const float t = state->t;
    if (blockIdx.x == 0 && threadIdx.x == 0) cp->t = t;  // the fill kernel reads t from here
    const size_t base = (size_t)blockIdx.x * TV_TILE;
    float4 v[TILE_U];
    load_tile<VEC>(src, n, base, 0xffffffffu, v);
    uint32_t q = 0, mx = 0;
#pragma unroll
    for (uint32_t u = 0; u < TILE_U; ++u) {
        const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float x = comp(v[u], j);
            const bool valid = e + j < n;
            const float ax = fabsf(x);
            if (valid) mx = max(mx, f2u(ax));
            if (valid && ax >= t) q |= 1u << (u * 4 + j);
        }
    }
    uint32_t slot[TILE_U * 4], total;
    tile_ranks(q, slot, s_wt, &total);
    if (q) {
#pragma unroll
        for (uint32_t u = 0; u < TILE_U; ++u) {
            const size_t e = base + 4 * ((size_t)u * STG_WG + threadIdx.x);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (((q >> (u * 4 + j)) & 1u) && slot[u * 4 + j] < TV_STAGE) {
                    const size_t o = (size_t)blockIdx.x * TV_STAGE + slot[u * 4 + j];
                    stage_pos[o] = (uint32_t)(e + j);
                    stage_val[o] = comp(v[u], j);
                }
            }
        }
    }
    mx = wave_max(mx);
    if (__lane_id() == 0) s_max[threadIdx.x >> 6] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) m = max(m, s_max[w]);
        tile_cnt[blockIdx.x] = total;
        tile_max[blockIdx.x] = m;
    }
}

struct TvFillArgs {
    const float *src;
    uint64_t n;
    uint32_t ntiles, k, cap;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    const CallParams *cp;
    const uint32_t *tile_cnt;
    const uint32_t *tile_max;
    const uint32_t *stage_pos;
    const float *stage_val;
};

template <bool VEC>
__global__ void __launch_bounds__(STG_WG) tv_fill(TvFillArgs a) {
    __shared__ uint64_t sh64[STG_WAVES];
    __shared__ uint32_t s_wt[TILE_U * STG_WAVES + 1];
    __shared__ uint32_t s_max[STG_WAVES];
    const uint32_t G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
    const uint32_t t_begin = (uint32_t)((uint64_t)w * a.ntiles / G);
    const uint32_t t_end = (uint32_t)((uint64_t)(w + 1) * a.ntiles / G);
    const float t = a.cp->t;  // the state slot itself is rewritten by workgroup 0 below

    uint64_t tot = 0, bef = 0;
    uint32_t mx = 0;
    for (uint32_t i = tid; i < a.ntiles; i += STG_WG) {
        const uint32_t c = a.tile_cnt[i];
        tot += c;
        if (i < t_begin) bef += c;
        if (w == 0) mx = max(mx, a.tile_max[i]);
    }
    const uint64_t cnt = wg_sum64(tot, sh64);
    uint64_t P = wg_sum64(bef, sh64);

    for (uint32_t tile = t_begin; tile < t_end && P < a.cap; ++tile) {
        const uint32_t c = a.tile_cnt[tile];
        const uint32_t m = (uint32_t)std::min<uint64_t>(c, a.cap - P);
        if (c <= TV_STAGE) {
            for (uint32_t i = tid; i < m; i += STG_WG) {
                a.idx[P + i] = a.stage_pos[(size_t)tile * TV_STAGE + i];
                a.val[P + i] = a.stage_val[(size_t)tile * TV_STAGE + i];
            }
        } else {  // staging overflowed: re-derive this tile's ranks from src
            float4 v[TILE_U];
            const size_t base = (size_t)tile * TV_TILE;
            load_tile<VEC>(a.src, a.n, base, 0xffffffffu, v);
            uint32_t q = 0;
#pragma unroll
            for (uint32_t u = 0; u < TILE_U; ++u) {
                const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (e + j < a.n && fabsf(comp(v[u], j)) >= t) q |= 1u << (u * 4 + j);
            }
            uint32_t slot[TILE_U * 4], total;
            tile_ranks(q, slot, s_wt, &total);
#pragma unroll
            for (uint32_t u = 0; u < TILE_U; ++u) {
                const size_t e = base + 4 * ((size_t)u * STG_WG + tid);
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (((q >> (u * 4 + j)) & 1u) && slot[u * 4 + j] < m) {
                        a.idx[P + slot[u * 4 + j]] = (uint32_t)(e + j);
                        a.val[P + slot[u * 4 + j]] = comp(v[u], j);
                    }
            }
        }
        P += c;
    }

    if (w == 0) {
        mx = wave_max(mx);
        if (__lane_id() == 0) s_max[tid >> 6] = mx;
        __syncthreads();
        if (tid == 0) {
            uint32_t g = 0;
            for (uint32_t i = 0; i < STG_WAVES; ++i) g = max(g, s_max[i]);
            const float gmax = a.n ? u2f(g) : -1.f;
            float nt = t;
            if ((uint64_t)a.k > cnt) nt = (float)((double)t * 0.99);
            else if ((uint64_t)a.k < cnt) nt = (float)fma(0.01 * (double)cnt / (double)a.k, (double)gmax, (double)t);
            a.state->t = nt;
            a.state->init = 1;
            *a.count_out = (uint32_t)std::min<uint64_t>(cnt, a.cap);
        }
    }
}

}  // namespace

hipError_t launch_tv(const TvLaunch &a, const DevWS &ws, hipStream_t s) {
    const uint32_t ntiles = (uint32_t)((a.n + TV_TILE - 1) / TV_TILE);
    if (a.first) {
        const uint32_t rank = (uint32_t)std::min<uint64_t>(a.k, a.n - 1);
        hipError_t e = launch_radix_select(a.src, a.n, 0xffffffffu, 0, nullptr, rank, ws, a.num_cu, s);
        if (e != hipSuccess) return e;
        tv_init_state<<<1, 1, 0, s>>>(a.state, ws.rsel);
    }
    if (a.ev) (void)hipEventRecord(a.ev[0], s);
    const bool vec = (reinterpret_cast<uintptr_t>(a.src) & 15u) == 0;
    if (vec) tv_scan<true><<<ntiles, STG_WG, 0, s>>>(a.src, a.n, a.state, ws.tile_cnt, ws.tile_aux, ws.stage_pos, ws.stage_val, ws.cp);
    else tv_scan<false><<<ntiles, STG_WG, 0, s>>>(a.src, a.n, a.state, ws.tile_cnt, ws.tile_aux, ws.stage_pos, ws.stage_val, ws.cp);
    TvFillArgs f;
    f.src = a.src;
    f.n = a.n;
    f.ntiles = ntiles;
    f.k = a.k;
    f.cap = a.cap;
    f.idx = a.idx;
    f.val = a.val;
    f.count_out = a.count_out;
    f.state = a.state;
    f.cp = ws.cp;
    f.tile_cnt = ws.tile_cnt;
    f.tile_max = ws.tile_aux;
    f.stage_pos = ws.stage_pos;
    f.stage_val = ws.stage_val;
    const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)a.num_cu, ntiles));
    if (a.ev) (void)hipEventRecord(a.ev[1], s);
    if (vec) tv_fill<true><<<G, STG_WG, 0, s>>>(f);
    else tv_fill<false><<<G, STG_WG, 0, s>>>(f);
    if (a.ev) (void)hipEventRecord(a.ev[2], s);
    return hipGetLastError();
}

}  // namespace stg
