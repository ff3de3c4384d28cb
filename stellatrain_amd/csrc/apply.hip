// apply.hip -- inverse path of config 5: MERGE decompress + sparse SGD (gfx950).
//
// MERGE decompress: engine/modules/cpu_optimize.cpp:40-72.  For each of
// `world` rank streams: tmp = zeros(n); tmp.index_put_(idx_r, val_r);
// merged += tmp (rank order); merged /= float(world); the output is merged
// gathered at the union of the indices.  Within a rank the codec's indices
// are unique, so a plain (non-atomic) add per rank, launched in rank order,
// reproduces the rank-ordered float sum exactly (adding the +0.0 of ranks that
// miss an index never changes a finite sum; the first add maps -0.0 to +0.0
// exactly as 0 + v does).  The output is index-ascending (the reference's
// unordered_set order is unspecified and SGD is per-index).  world == 1 needs
// no dense scratch: out = (0.0f + v) / 1.0f in stream order.
//
// Duplicate indices within a rank (the wire format's signed u16 saturation
// maps every index >= 32768 of an 8-wide block to 32767, comm_manager.cpp:
// 509-529): index_put_ without accumulate keeps the LAST occurrence (the
// reference's per-rank CPU index_put_ runs sequentially at these sizes), and
// unique1d (:14-24) leaves one entry per index.  Every rank therefore first
// elects its winner per index (atomicMax of position + 1 into a u32 scratch
// that is zero between calls), and only the winner scatters (and re-zeroes the
// scratch word); world == 1 keeps the winners in stream order.
//
// Sparse SGD: optim/sgd.cpp:34-55 and the scalar loop :221-263 with the FMA
// shapes GCC -O3 -march=broadwell emits (read from the object code):
//   wd:        g = fmaf(wd, x, g)                        (vfmadd231ss, :235)
//   momentum:  b = first ? g : fmaf(b_old, m, (1-d)*g)   (vfmadd231ss, :242)
//   nesterov:  g = fmaf(m, b, g)  else g = b             (vfmadd231ss, :247)
//   update:    x = (float)fma(-lr, (double)g, (double)x) (vfnmadd231sd, :256)
//
// Sparse Adam: optim/adam.cpp:19-86, shapes from the -O3 object code (see
// oracle/stg_oracle.cpp adam_apply for the derivation):
//   g = maximize ? -g : g;  wd: g = fmaf(wd, x, g)
//   mt = fmaf(b1, m, (1-b1)*g);  vt = fmaf(b2, v, ((1-b2)*g)*g)           (float)
//   x' = (float)(x - (mt/c1)*lr / den),  den = eps + sqrt(vt/c2)          (double)
//   amsgrad: den = (double)(sqrtf(vmax_i) + eps), vmax_i the running max over
//   the call's elements in stream order of (float)(vt/c2) (adam.cpp:71) -- a
//   prefix max: one launch, each 1,024-element tile publishes its maximum as a
//   tagged word and takes the maximum over its predecessors' words
//   (decoupled look-back; max needs no inclusive chain), then applies.
//   Indices are unique within a call (codec output / MERGE union), so the
//   elements are independent apart from vmax.
#include <algorithm>
#include <cstdlib>

#include "ws.h"

namespace stg {

namespace {

constexpr uint32_t MARK_TILE = MERGE_TILE;  // marks (or pairs) per tile (one uint4 of marks per lane)

// Winner election: win[j] = 1 + the last position of index j in the rank's
// stream (indices >= n are dropped: the reference would throw on them).
// With `dup` (world 1): any repeated or out-of-range index sets it (the
// emission then elects; otherwise every pair is its index's only occurrence and
// the emission copies the stream), and the emission's tile ticket starts at 0.
__global__ void __launch_bounds__(STG_WG) win_mark(const uint32_t *__restrict__ idx, size_t m, size_t n,
                                                   uint32_t *__restrict__ win, uint32_t *dup, uint64_t *ticket) {
    if (ticket && blockIdx.x == 0 && threadIdx.x == 0) st_sc1(ticket, 0ull);
    const size_t stride = (size_t)gridDim.x * STG_WG;
    for (size_t i = (size_t)blockIdx.x * STG_WG + threadIdx.x; i < m; i += stride) {
        const uint32_t j = idx[i];
        if (!dup) {
            if (j < n) atomicMax(&win[j], (uint32_t)i + 1u);
        } else if (j >= n || atomicMax(&win[j], (uint32_t)i + 1u) != 0u) {
            g_or(dup, 1u);  // rare for codec output: its indices are unique
        }
    }
}

// world == 1, pass 1: winners per tile of MARK_TILE pairs.
__global__ void __launch_bounds__(STG_WG) win_count(const uint32_t *__restrict__ idx, size_t m, size_t n,
                                                    const uint32_t *__restrict__ win, uint32_t *__restrict__ tile_cnt);
// world == 1, pass 2: ordered compaction of the winners (look-up of the
// earlier tiles' counts), re-zeroing their scratch words.
__global__ void __launch_bounds__(STG_WG) win_emit1(const uint32_t *__restrict__ idx, const float *__restrict__ val,
                                                    size_t m, size_t n, uint32_t ntiles, uint32_t *__restrict__ win,
                                                    const uint32_t *__restrict__ tile_cnt,
                                                    uint32_t *__restrict__ out_idx, float *__restrict__ out_val,
                                                    uint32_t *out_count);

// world > 1: rank r's scatter and rank r+1's winner election in one launch,
// on the two halves of the election scratch (rank parity), so a rank's
// election never sees the previous rank's words: threads [0, m) scatter rank
// `sr` (if any), threads [m, 2m) elect rank `mr` (if any).
__global__ void __launch_bounds__(STG_WG) scatter_mark(const uint32_t *__restrict__ sidx, const float *__restrict__ sval,
                                                       uint32_t *__restrict__ swin, const uint32_t *__restrict__ midx,
                                                       uint32_t *__restrict__ mwin, size_t m, size_t n,
                                                       float *__restrict__ dense, uint8_t *__restrict__ mark) {
    const size_t stride = (size_t)gridDim.x * STG_WG;
    for (size_t t = (size_t)blockIdx.x * STG_WG + threadIdx.x; t < 2 * m; t += stride) {
        if (t < m) {
            if (!sidx) continue;
            const uint32_t j = sidx[t];
            if (j >= n || swin[j] != (uint32_t)t + 1u) continue;  // a later occurrence wins
            swin[j] = 0;
            dense[j] += sval[t];
            mark[j] = 1;
        } else {
            if (!midx) continue;
            const size_t i = t - m;
            const uint32_t j = midx[i];
            if (j < n) atomicMax(&mwin[j], (uint32_t)i + 1u);
        }
    }
}

__device__ __forceinline__ uint32_t nz_bytes(uint32_t w) {
    uint32_t c = 0;
    c += (w & 0xffu) != 0;
    c += (w & 0xff00u) != 0;
    c += (w & 0xff0000u) != 0;
    c += (w & 0xff000000u) != 0;
    return c;
}

__device__ __forceinline__ uint4 load_marks(const uint8_t *mark, size_t n, size_t e) {
    if (e + 16 <= n) return *reinterpret_cast<const uint4 *>(mark + e);
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t b = 0; b < 16; ++b)
        if (e + b < n) w[b >> 2] |= (uint32_t)mark[e + b] << (8 * (b & 3));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void __launch_bounds__(STG_WG) mark_count(const uint8_t *__restrict__ mark, size_t n,
                                                     uint32_t *__restrict__ tile_cnt) {
    __shared__ uint32_t s[STG_WAVES];
    const size_t e = (size_t)blockIdx.x * MARK_TILE + 16 * threadIdx.x;
    const uint4 v = load_marks(mark, n, e);
    uint32_t c = nz_bytes(v.x) + nz_bytes(v.y) + nz_bytes(v.z) + nz_bytes(v.w);
    c = wave_sum(c);
    if (__lane_id() == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) t += s[w];
        tile_cnt[blockIdx.x] = t;
    }
}

// Exclusive prefixes of the per-tile mark counts at [ntiles + t] and the total
// in *out_count (one 1024-thread workgroup, 4 tiles per thread per round).
__global__ void __launch_bounds__(1024) mark_scan(uint32_t *__restrict__ tile_cnt, uint32_t ntiles,
                                                  uint32_t *out_count) {
    __shared__ uint32_t sh[16 + 1];
    uint32_t run = 0;
    for (uint32_t t0 = 0; t0 < ntiles; t0 += 4 * 1024) {
        const uint32_t tb = t0 + 4 * threadIdx.x;
        uint32_t c[4], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) { c[q] = tb + q < ntiles ? tile_cnt[tb + q] : 0u; sum += c[q]; }
        uint32_t tot;
        uint32_t p = run + blk_excl_scan<16>(sum, sh, &tot);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q)
            if (tb + q < ntiles) { tile_cnt[ntiles + tb + q] = p; p += c[q]; }
        run += tot;
    }
    if (threadIdx.x == 0) *out_count = run;
}

// One workgroup per tile of MARK_TILE marks: the marked indices in order at
// the tile's prefix, value dense / world; dense and marks zeroed behind it.
// A lane's 16 marks and 16 dense values are one uint4 and four float4 loads.
__global__ void __launch_bounds__(STG_WG) mark_emit_tile(uint8_t *__restrict__ mark, float *__restrict__ dense,
                                                         size_t n, uint32_t ntiles, float world,
                                                         const uint32_t *__restrict__ tile_cnt,
                                                         uint32_t *__restrict__ out_idx, float *__restrict__ out_val) {
    __shared__ uint32_t sh[STG_WAVES + 1];
    const uint32_t tile = blockIdx.x, tid = threadIdx.x;
    if (!tile_cnt[tile]) return;  // uniform: nothing marked in this tile
    const uint64_t P = tile_cnt[ntiles + tile];
    const size_t e = (size_t)tile * MARK_TILE + 16 * tid;
    const uint4 v = load_marks(mark, n, e);
    const uint32_t words[4] = {v.x, v.y, v.z, v.w};
    const uint32_t c = nz_bytes(v.x) + nz_bytes(v.y) + nz_bytes(v.z) + nz_bytes(v.w);
    const bool full = e + 16 <= n;
    float d[16];
    if (c && full) {
        const float4 *p = reinterpret_cast<const float4 *>(dense + e);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            const float4 x = p[q];
            d[4 * q] = x.x; d[4 * q + 1] = x.y; d[4 * q + 2] = x.z; d[4 * q + 3] = x.w;
        }
    }
    uint32_t tc;
    uint32_t r = wg_excl_scan(c, sh, &tc);
    if (!c) return;
#pragma unroll
    for (uint32_t b = 0; b < 16; ++b) {
        if ((words[b >> 2] >> (8 * (b & 3))) & 0xffu) {
            const size_t j = e + b;
            out_idx[P + r] = (uint32_t)j;
            out_val[P + r] = (full ? d[b] : dense[j]) / world;
            if (!full) { dense[j] = 0.f; mark[j] = 0; }
            ++r;
        }
    }
    if (full) {  // leave the scratch zeroed for the next call
        float4 *p = reinterpret_cast<float4 *>(dense + e);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) p[q] = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<uint4 *>(mark + e) = make_uint4(0u, 0u, 0u, 0u);
    }
}


constexpr uint32_t WPER = MARK_TILE / STG_WG;  // 16 consecutive pairs per lane
static_assert(WPER == 16, "four uint4 of indices per lane");

// The lane's 16 pairs e .. e+15: their indices, and which of them win (bit b).
// Every load is issued before any is used -- the 16 index loads together,
// then the 16 winner words (clamped addresses, results masked) -- two round
// trips per lane instead of 32 dependent ones.
template <uint32_t WP>
__device__ __forceinline__ uint32_t win_keep_t(const uint32_t *__restrict__ idx, size_t m, size_t n,
                                               const uint32_t *__restrict__ win, size_t e, uint32_t (&j)[WP]) {
    if (WP % 4 == 0 && e + WP <= m && (reinterpret_cast<uintptr_t>(idx + e) & 15u) == 0) {
        const uint4 *p = reinterpret_cast<const uint4 *>(idx + e);
#pragma unroll
        for (uint32_t q = 0; q < WP / 4; ++q) {
            const uint4 v = p[q];
            j[4 * q] = v.x; j[4 * q + 1] = v.y; j[4 * q + 2] = v.z; j[4 * q + 3] = v.w;
        }
    } else {
#pragma unroll
        for (uint32_t b = 0; b < WP; ++b) j[b] = idx[std::min<size_t>(e + b, m - 1)];
    }
    uint32_t w[WP];
#pragma unroll
    for (uint32_t b = 0; b < WP; ++b) w[b] = win[j[b] < n ? j[b] : 0u];
    uint32_t keep = 0;
#pragma unroll
    for (uint32_t b = 0; b < WP; ++b)
        if (e + b < m && j[b] < n && w[b] == (uint32_t)(e + b) + 1u) keep |= 1u << b;
    return keep;
}
__device__ __forceinline__ uint32_t win_keep(const uint32_t *__restrict__ idx, size_t m, size_t n,
                                             const uint32_t *__restrict__ win, size_t e, uint32_t (&j)[WPER]) {
    return win_keep_t<WPER>(idx, m, n, win, e, j);
}

__global__ void __launch_bounds__(STG_WG) win_count(const uint32_t *__restrict__ idx, size_t m, size_t n,
                                                    const uint32_t *__restrict__ win, uint32_t *__restrict__ tile_cnt) {
    __shared__ uint32_t s[STG_WAVES];
    const size_t e = (size_t)blockIdx.x * MARK_TILE + (size_t)WPER * threadIdx.x;
    uint32_t j[WPER];
    uint32_t c = e < m ? (uint32_t)__popc(win_keep(idx, m, n, win, e, j)) : 0u;
    c = wave_sum(c);
    if (__lane_id() == 0) s[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t w = 0; w < STG_WAVES; ++w) t += s[w];
        tile_cnt[blockIdx.x] = t;
    }
}

__global__ void __launch_bounds__(STG_WG) win_emit1(const uint32_t *__restrict__ idx, const float *__restrict__ val,
                                                    size_t m, size_t n, uint32_t ntiles, uint32_t *__restrict__ win,
                                                    const uint32_t *__restrict__ tile_cnt,
                                                    uint32_t *__restrict__ out_idx, float *__restrict__ out_val,
                                                    uint32_t *out_count) {
    __shared__ uint64_t sh64[STG_WAVES];
    __shared__ uint32_t sh[STG_WAVES + 1];
    const uint32_t G = gridDim.x, w = blockIdx.x, tid = threadIdx.x;
    const uint32_t t_begin = (uint32_t)((uint64_t)w * ntiles / G);
    const uint32_t t_end = (uint32_t)((uint64_t)(w + 1) * ntiles / G);
    uint64_t tot = 0, bef = 0;
    for (uint32_t i = tid; i < ntiles; i += STG_WG) {
        const uint32_t c = tile_cnt[i];
        tot += c;
        if (i < t_begin) bef += c;
    }
    const uint64_t total = wg_sum64(tot, sh64);
    uint64_t P = wg_sum64(bef, sh64);
    for (uint32_t tile = t_begin; tile < t_end; ++tile) {
        const size_t e = (size_t)tile * MARK_TILE + (size_t)WPER * tid;
        uint32_t j[WPER];
        const uint32_t keep = e < m ? win_keep(idx, m, n, win, e, j) : 0u;
        float v[WPER];  // the values, loaded alongside (clamped addresses)
        if (e + WPER <= m && (reinterpret_cast<uintptr_t>(val + e) & 15u) == 0) {
            const float4 *p = reinterpret_cast<const float4 *>(val + e);
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                const float4 x = p[q];
                v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
            }
        } else {
#pragma unroll
            for (uint32_t b = 0; b < WPER; ++b) v[b] = m ? val[std::min<size_t>(e + b, m - 1)] : 0.f;
        }
        uint32_t tc;
        uint32_t r = wg_excl_scan((uint32_t)__popc(keep), sh, &tc);
#pragma unroll
        for (uint32_t b = 0; b < WPER; ++b) {
            if (keep >> b & 1u) {
                out_idx[P + r] = j[b];
                out_val[P + r] = (0.0f + v[b]) / 1.0f;
                win[j[b]] = 0;  // scratch back to zero for the next call
                ++r;
            }
        }
        P += tc;
    }
    if (w == 0 && tid == 0) *out_count = (uint32_t)total;
}

// world == 1 in one launch after win_mark: tiles in ticket order (a workgroup
// only waits on tiles taken before its own, so no co-residency is needed);
// each publishes its winner count as a tagged word, sums the earlier tiles'
// counts (look-back) and writes its winners at that offset; the last tile
// writes the count.
// SGD::optimize_raw on one element (optim/sgd.cpp:34-263, scalar path), with
// param[id] = x and mom[id] = m loaded by the caller: the same expression as
// sgd_apply, so a step fused into the emission agrees with it bitwise.
__device__ __forceinline__ void sgd_step(const SgdLaunch &a, uint32_t id, float g, float x, float m) {
    if (a.weight_decay != 0.f) g = fmaf(a.weight_decay, x, g);
    if (a.mom) {
        const float b = a.first ? g : fmaf(m, a.momentum, (1.0f - a.dampening) * g);
        g = a.nesterov ? fmaf(a.momentum, b, g) : b;
        a.mom[id] = b;
    }
    a.param[id] = (float)fma(-a.lr, (double)g, (double)x);
}

// Adam::optimize_raw on one element (optim/adam.cpp:19-86, no amsgrad), with
// param[id] = x, m[id] = m0, v[id] = v0 loaded by the caller: the expressions of
// adam_elem / adam_apply below, so a fused step agrees with them bitwise.
__device__ __forceinline__ void adam_step(const AdamLaunch &a, uint32_t id, float g, float x, float m0, float v0) {
    if (a.maximize) g = -g;
    if (a.weight_decay != 0.f) g = fmaf(a.weight_decay, x, g);
    const float mt = fmaf(a.b1, m0, (1.f - a.b1) * g);
    const float vt = fmaf(a.b2, v0, ((1.f - a.b2) * g) * g);
    const double num = ((double)mt / a.c1) * a.lr;
    const double vt_hat = (double)vt / a.c2;
    a.param[id] = (float)((double)x - num / ((double)a.eps + sqrt(vt_hat)));
    a.m[id] = mt;
    a.v[id] = vt;
}

struct Win1Args {
    const uint32_t *idx;
    const float *val;
    size_t m, n;
    uint32_t ntiles;
    uint32_t *win;
    uint64_t *desc;     // per tile: {call tag:32 | winners:32}
    uint64_t *ticket;   // tiles taken, monotonic over the scratch's calls (zero at creation)
    uint64_t base;      // its value when this call starts
    uint32_t tag;       // this call's tag, >= 1
    uint32_t *out_idx;
    float *out_val;
    uint32_t *out_count;
    uint32_t *fail;     // [0] sticky failure bits (a tile whose look-back gave up); [1] the tag of the last call that did
    uint32_t *dup;      // set by win_mark when an index repeats (or is >= n); zeroed by the last tile then
    bool fuse_sgd;      // ModuleCpuOptimize::run: optimize_raw on every winner as it is emitted
    SgdLaunch sgd;
    bool fuse_adam;     // ... with Adam (no amsgrad)
    AdamLaunch adam;
};

// WP pairs per lane: 4 (the default; 1,024-pair tiles, four times the
// workgroups and the gathers of 16) or 16 (4,096-pair tiles: 41 workgroups at
// 167,772 pairs, 13 us per call in the C5 kernel trace).
template <uint32_t WP>
__global__ void __launch_bounds__(STG_WG) win_emit1t(Win1Args a) {
    __shared__ uint32_t sh[STG_WAVES + 1];
    __shared__ uint32_t s_tile, s_bad;
    __shared__ uint64_t s_P, s_psum[STG_WAVES];
    __shared__ uint32_t s_dup;
    const uint32_t tid = threadIdx.x, lane = __lane_id();
    if (tid == 0) s_dup = ld_sc1(a.dup);
    __syncthreads();
    if (!s_dup) {
        // no index repeats: every pair wins and keeps its place, so the output
        // is the stream itself -- no ticket, no look-back (tile = block)
        const size_t e = (size_t)blockIdx.x * (WP * STG_WG) + (size_t)WP * tid;
        uint32_t j[WP];
        float v[WP];
        if (WP % 4 == 0 && e + WP <= a.m && (reinterpret_cast<uintptr_t>(a.idx + e) & 15u) == 0 &&
            (reinterpret_cast<uintptr_t>(a.val + e) & 15u) == 0) {
#pragma unroll
            for (uint32_t q = 0; q < WP / 4; ++q) {
                const uint4 x = reinterpret_cast<const uint4 *>(a.idx + e)[q];
                const float4 y = reinterpret_cast<const float4 *>(a.val + e)[q];
                j[4 * q] = x.x; j[4 * q + 1] = x.y; j[4 * q + 2] = x.z; j[4 * q + 3] = x.w;
                v[4 * q] = y.x; v[4 * q + 1] = y.y; v[4 * q + 2] = y.z; v[4 * q + 3] = y.w;
            }
        } else {
#pragma unroll
            for (uint32_t b = 0; b < WP; ++b) {
                const size_t i = std::min<size_t>(e + b, a.m ? a.m - 1 : 0);
                j[b] = a.idx[i];
                v[b] = a.val[i];
            }
        }
        float xp[WP], mp[WP], vp[WP];
        if (a.fuse_sgd) {  // every pair is a winner: its parameter and momentum words, loaded together
#pragma unroll
            for (uint32_t b = 0; b < WP; ++b) {
                const uint32_t id = e + b < a.m ? j[b] : 0u;
                xp[b] = a.sgd.param[id];
                mp[b] = a.sgd.mom ? a.sgd.mom[id] : 0.f;
            }
        } else if (a.fuse_adam) {
#pragma unroll
            for (uint32_t b = 0; b < WP; ++b) {
                const uint32_t id = e + b < a.m ? j[b] : 0u;
                xp[b] = a.adam.param[id];
                mp[b] = a.adam.m[id];
                vp[b] = a.adam.v[id];
            }
        }
#pragma unroll
        for (uint32_t b = 0; b < WP; ++b) {
            if (e + b < a.m) {
                const float g = (0.0f + v[b]) / 1.0f;  // merged_grad[j] (cpu_optimize.cpp:49-55), world 1
                a.out_idx[e + b] = j[b];
                a.out_val[e + b] = g;
                if (a.fuse_sgd) sgd_step(a.sgd, j[b], g, xp[b], mp[b]);  // indices unique: updates commute
                else if (a.fuse_adam) adam_step(a.adam, j[b], g, xp[b], mp[b], vp[b]);
                a.win[j[b]] = 0;  // scratch back to zero for the next call
            }
        }
        if (tid == 0 && blockIdx.x == a.ntiles - 1) {
            __builtin_amdgcn_s_waitcnt(0);
            *a.out_count = (uint32_t)a.m;  // no look-back in this call: nothing of it can have failed
        }
        return;
    }
    if (tid == 0) { s_tile = (uint32_t)(g_add(a.ticket, 1ull) - a.base); s_bad = 0; }
    __syncthreads();
    const uint32_t tile = s_tile;
    const size_t e = (size_t)tile * (WP * STG_WG) + (size_t)WP * tid;
    uint32_t j[WP];
    const uint32_t keep = e < a.m ? win_keep_t<WP>(a.idx, a.m, a.n, a.win, e, j) : 0u;
    float v[WP];
    if (WP % 4 == 0 && e + WP <= a.m && (reinterpret_cast<uintptr_t>(a.val + e) & 15u) == 0) {
        const float4 *p = reinterpret_cast<const float4 *>(a.val + e);
#pragma unroll
        for (uint32_t q = 0; q < WP / 4; ++q) {
            const float4 x = p[q];
            v[4 * q] = x.x; v[4 * q + 1] = x.y; v[4 * q + 2] = x.z; v[4 * q + 3] = x.w;
        }
    } else {
#pragma unroll
        for (uint32_t b = 0; b < WP; ++b) v[b] = a.m ? a.val[std::min<size_t>(e + b, a.m - 1)] : 0.f;
    }
    float xp[WP], mp[WP], vp[WP];
    if (a.fuse_sgd) {  // the winners' parameter and momentum words, loaded under the look-back
#pragma unroll
        for (uint32_t b = 0; b < WP; ++b) {
            const uint32_t id = (keep >> b & 1u) ? j[b] : 0u;
            xp[b] = a.sgd.param[id];
            mp[b] = a.sgd.mom ? a.sgd.mom[id] : 0.f;
        }
    } else if (a.fuse_adam) {
#pragma unroll
        for (uint32_t b = 0; b < WP; ++b) {
            const uint32_t id = (keep >> b & 1u) ? j[b] : 0u;
            xp[b] = a.adam.param[id];
            mp[b] = a.adam.m[id];
            vp[b] = a.adam.v[id];
        }
    }
    uint32_t tc;
    uint32_t r = wg_excl_scan((uint32_t)__popc(keep), sh, &tc);
    if (tid == 0) st_sc1(&a.desc[tile], ((uint64_t)a.tag << 32) | tc);
    {   // look-back over tiles 0 .. tile-1, STG_WG per round trip
        uint64_t Pl = 0;
        bool gave = false;
        for (uint32_t i0 = 0; i0 < tile; i0 += STG_WG) {
            const uint32_t i = i0 + tid;
            uint64_t d = i < tile ? ld_sc1(&a.desc[i]) : 0ull;
            uint64_t st = 0;
            for (uint32_t spins = 0; i < tile && (uint32_t)(d >> 32) != a.tag; ++spins) {
                __builtin_amdgcn_s_sleep(4);
                d = ld_sc1(&a.desc[i]);
                if (spin_expired(spins, st)) { gave = true; break; }  // 200 ms: give up, poison the count
            }
            Pl += (uint32_t)d;
        }
        if (gave) s_bad = 1;
        Pl = wave_sum64(Pl);
        if (lane == 0) s_psum[tid >> 6] = Pl;
        __syncthreads();
        if (tid == 0) {
            uint64_t t2 = 0;
            for (uint32_t w = 0; w < STG_WAVES; ++w) t2 += s_psum[w];
            s_P = t2;
        }
    }
    __syncthreads();
    const uint64_t P = s_P;
    const bool bad = s_bad != 0;
    // a tile that gave up has no valid offset: it writes nothing, marks the
    // scratch's sticky failure word (stg_scatter_merge_check) and, as the last
    // tile, poisons the count; the last tile also poisons it for any earlier
    // tile that gave up first
    if (bad && tid == 0) {
        g_or(a.fail, FAIL_SPIN_TIMEOUT);  // sticky, for stg_scatter_merge_check
        st_sc1(a.fail + 1, a.tag);        // this call's count is poisoned, later calls' are not
    }
#pragma unroll
    for (uint32_t b = 0; b < WP; ++b) {
        if (keep >> b & 1u) {
            const float g = (0.0f + v[b]) / 1.0f;
            if (!bad) {
                a.out_idx[P + r] = j[b];
                a.out_val[P + r] = g;
            }
            if (a.fuse_sgd) sgd_step(a.sgd, j[b], g, xp[b], mp[b]);  // each index elected once: updates commute
            else if (a.fuse_adam) adam_step(a.adam, j[b], g, xp[b], mp[b], vp[b]);
            a.win[j[b]] = 0;  // scratch back to zero for the next call
            ++r;
        }
    }
    if (tid == 0 && tile == a.ntiles - 1) {
        __builtin_amdgcn_s_waitcnt(0);
        *a.out_count = (bad || ld_sc1(a.fail + 1) == a.tag) ? 0xffffffffu : (uint32_t)(P + tc);
        // every tile read the flag before publishing its count (the look-back
        // above saw them all): clear it for the next call
        if (!bad) st_sc1(a.dup, 0u);
    }
}

// a device count of POISON_COUNT (a failed producer) is length 0: never step
// over slots nobody wrote
__device__ __forceinline__ uint32_t dev_len(uint32_t cap, const uint32_t *d_len) {
    if (!d_len) return cap;
    const uint32_t c = *d_len;
    return c == POISON_COUNT ? 0u : min(cap, c);
}

__global__ void __launch_bounds__(STG_WG) sgd_apply(SgdLaunch a) {
    const uint32_t len = dev_len(a.grad_len, a.d_grad_len);
    const uint32_t stride = gridDim.x * STG_WG;
    for (uint32_t i = blockIdx.x * STG_WG + threadIdx.x; i < len; i += stride) {
        const uint32_t id = a.gidx[i];
        if (id >= a.param_len) continue;  // an index past the parameter (bad input): never written
        const float x = a.param[id];
        float g = a.grad[i];
        if (a.weight_decay != 0.f) g = fmaf(a.weight_decay, x, g);
        if (a.mom) {
            const float b = a.first ? g : fmaf(a.mom[id], a.momentum, (1.0f - a.dampening) * g);
            g = a.nesterov ? fmaf(a.momentum, b, g) : b;
            a.mom[id] = b;
        }
        a.param[id] = (float)fma(-a.lr, (double)g, (double)x);
    }
}

// Error feedback (compress.cpp:172-186): the bucket, with every selected
// index zeroed, becomes the residual -- and the bucket itself is left zeroed
// at those indices, as the reference's in-place src[idx[i]] = 0 leaves it.
// Pass 1 streams grad -> residual (float4, nontemporal); pass 2 zeroes both
// arrays at the numel indices (slots past the count hold index 0, so
// element 0 is zeroed too, as in the reference).
__global__ void __launch_bounds__(STG_WG) ef_copy(const float *__restrict__ grad, float *__restrict__ resid,
                                                  size_t n) {
    const size_t n4 = n / 4;
    const size_t stride = (size_t)gridDim.x * STG_WG;
    typedef float f4v __attribute__((ext_vector_type(4)));
    const f4v *g4 = reinterpret_cast<const f4v *>(grad);
    f4v *r4 = reinterpret_cast<f4v *>(resid);
    constexpr uint32_t UF = 4;
    for (size_t i0 = (size_t)blockIdx.x * STG_WG + threadIdx.x; i0 < n4; i0 += UF * stride) {
        f4v v[UF];
#pragma unroll
        for (uint32_t u = 0; u < UF; ++u) {
            const size_t i = i0 + u * stride;
            if (i < n4) v[u] = __builtin_nontemporal_load(g4 + i);
        }
#pragma unroll
        for (uint32_t u = 0; u < UF; ++u) {
            const size_t i = i0 + u * stride;
            if (i < n4) __builtin_nontemporal_store(v[u], r4 + i);
        }
    }
    if (blockIdx.x == 0)
        for (size_t i = n4 * 4 + threadIdx.x; i < n; i += STG_WG) resid[i] = grad[i];
}

__global__ void __launch_bounds__(STG_WG) ef_zero(float *__restrict__ grad, float *__restrict__ resid,
                                                  const uint32_t *__restrict__ idx, size_t numel, size_t n) {
    for (size_t j = (size_t)blockIdx.x * STG_WG + threadIdx.x; j < numel; j += (size_t)gridDim.x * STG_WG) {
        const uint32_t i = idx[j];
        if (i < n) {
            grad[i] = 0.f;
            resid[i] = 0.f;
        }
    }
}

struct AdamElem {
    float mt, vt;
    double num, vt_hat;
};

__device__ __forceinline__ AdamElem adam_elem(const AdamLaunch &a, float x, float g, uint32_t id) {
    if (a.maximize) g = -g;
    if (a.weight_decay != 0.f) g = fmaf(a.weight_decay, x, g);
    AdamElem e;
    e.mt = fmaf(a.b1, a.m[id], (1.f - a.b1) * g);
    e.vt = fmaf(a.b2, a.v[id], ((1.f - a.b2) * g) * g);
    e.num = ((double)e.mt / a.c1) * a.lr;
    e.vt_hat = (double)e.vt / a.c2;
    return e;
}

__device__ __forceinline__ uint32_t adam_len(const AdamLaunch &a) { return dev_len(a.grad_len, a.d_grad_len); }

__global__ void __launch_bounds__(STG_WG) adam_apply(AdamLaunch a) {
    const uint32_t len = adam_len(a);
    const uint32_t stride = gridDim.x * STG_WG;
    for (uint32_t i = blockIdx.x * STG_WG + threadIdx.x; i < len; i += stride) {
        const uint32_t id = a.gidx[i];
        if (id >= a.param_len) continue;  // an index past the parameter (bad input): never written
        adam_step(a, id, a.grad[i], a.param[id], a.m[id], a.v[id]);
    }
}

// amsgrad running max in the order-preserving uint map (0 = "no element": NaN
// vt_hat never wins the reference's vt_hat > vmax test).
__device__ __forceinline__ uint32_t ams_key(double vt_hat) {
    return vt_hat == vt_hat ? ford((float)vt_hat) : 0u;
}
__device__ __forceinline__ float ams_unkey(uint32_t k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
    const uint32_t lane = __lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (lane >= (uint32_t)d) v = max(v, o);
    }
    return v;
}

// One launch.  Tile t (ADAM_TILE consecutive elements of the call, lane l
// holds 4 consecutive ones) computes its elements, publishes its maximum key
// as (tag << 32 | key) in tiles[t] -- tag = the name's tick, so words of
// earlier calls never match -- and then reads tiles[0..t-1]: the running vmax
// before the tile is the maximum of the name's vmax and those words (max is
// idempotent, so no inclusive prefix chain is needed).  Predecessors have
// lower block ids, so they are dispatched first and always finish publishing;
// the poll is still bounded.  The last tile stores the call's vmax.
__global__ void __launch_bounds__(STG_WG) adam_apply_ams(AdamLaunch a, uint32_t tag) {
    __shared__ uint32_t sh[STG_WAVES], s_lb[STG_WAVES];
    __shared__ uint32_t s_pre;
    const uint32_t len = adam_len(a);
    const uint32_t ntile = (len + ADAM_TILE - 1) / ADAM_TILE;
    const uint32_t tile = blockIdx.x;
    if (tile >= ntile) return;
    const uint32_t base = tile * ADAM_TILE + threadIdx.x * 4;
    const uint32_t vmax0 = ford(*a.vmax);  // read before publishing: the last tile rewrites it
    uint32_t id[4], key[4];
    float x[4];
    AdamElem e[4];
    uint32_t run = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t i = base + j;
        key[j] = 0;
        id[j] = 0;
        x[j] = 0.f;
        e[j] = AdamElem{0.f, 0.f, 0.0, 0.0};
        if (i < len && a.gidx[i] < a.param_len) {  // an index past the parameter (bad input): skipped
            id[j] = a.gidx[i];
            x[j] = a.param[id[j]];
            e[j] = adam_elem(a, x[j], a.grad[i], id[j]);
            key[j] = ams_key(e[j].vt_hat);
        }
        run = max(run, key[j]);
    }
    const uint32_t inc = wave_incl_max(run);
    if (__lane_id() == 63) sh[threadIdx.x >> 6] = inc;
    __syncthreads();
    uint32_t tile_max = 0;
    for (uint32_t w = 0; w < STG_WAVES; ++w) tile_max = max(tile_max, sh[w]);
    uint64_t *words = reinterpret_cast<uint64_t *>(a.tiles);
    if (threadIdx.x == 0) st_sc1(&words[tile], ((uint64_t)tag << 32) | tile_max);
    // look-back by the whole workgroup: STG_WG predecessors per round trip
    {
        uint32_t pt = vmax0;
        for (uint32_t p = threadIdx.x; p < tile; p += STG_WG) {
            uint64_t w = ld_sc1(&words[p]);
            uint64_t st = 0;
            for (uint32_t spins = 0; (uint32_t)(w >> 32) != tag; ++spins) {
                if (spin_expired(spins, st)) {  // starved predecessor: flag it (stg_adam_check), never use a stale word silently
                    g_or(a.fail, FAIL_SPIN_TIMEOUT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                w = ld_sc1(&words[p]);
            }
            pt = max(pt, (uint32_t)w);
        }
        pt = wave_max(pt);
        if (__lane_id() == 0) s_lb[threadIdx.x >> 6] = pt;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t m = 0;
            for (uint32_t w = 0; w < STG_WAVES; ++w) m = max(m, s_lb[w]);
            s_pre = m;
        }
    }
    __syncthreads();
    uint32_t pre = s_pre;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) pre = max(pre, sh[w]);
    pre = max(pre, (uint32_t)__shfl_up(inc, 1, 64) * (__lane_id() != 0));
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
        const uint32_t i = base + j;
        pre = max(pre, key[j]);
        if (i < len && a.gidx[i] < a.param_len) {
            const float vm = ams_unkey(pre);
            a.param[id[j]] = (float)((double)x[j] - e[j].num / (double)(sqrtf(vm) + a.eps));
            a.m[id[j]] = e[j].mt;
            a.v[id[j]] = e[j].vt;
        }
    }
    if (tile == ntile - 1 && threadIdx.x == STG_WG - 1) *a.vmax = ams_unkey(pre);
}

}  // namespace

hipError_t launch_ef_zero(float *grad, float *resid, const uint32_t *idx, size_t numel, size_t n, int num_cu,
                          hipStream_t s) {
    if (!numel) return hipSuccess;
    const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>((numel + STG_WG - 1) / STG_WG,
                                                                          (size_t)num_cu * 4));
    ef_zero<<<blocks, STG_WG, 0, s>>>(grad, resid, idx, numel, n);
    return hipGetLastError();
}

hipError_t launch_error_feedback(float *grad, size_t n, const uint32_t *idx, size_t numel, float *resid, int num_cu,
                                 hipStream_t s) {
    if (n) {
        const bool vec = ((reinterpret_cast<uintptr_t>(grad) | reinterpret_cast<uintptr_t>(resid)) & 15u) == 0;
        const size_t work = vec ? (n / 4 + STG_WG - 1) / STG_WG : 0;
        const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>(work, (size_t)num_cu * 8));
        if (vec) ef_copy<<<blocks, STG_WG, 0, s>>>(grad, resid, n);
        else {
            const hipError_t e = hipMemcpyAsync(resid, grad, n * sizeof(float), hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return e;
        }
    }
    if (numel) {
        const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>((numel + STG_WG - 1) / STG_WG,
                                                                              (size_t)num_cu * 4));
        ef_zero<<<blocks, STG_WG, 0, s>>>(grad, resid, idx, numel, n);
    }
    return hipGetLastError();
}

hipError_t launch_scatter_merge(const uint32_t *idx, const float *val, size_t per_rank, int world, size_t n,
                                float *dense, uint8_t *mark, uint32_t *out_idx, float *out_val,
                                uint32_t *out_count, uint32_t *scratch_tiles, uint32_t *win, int num_cu,
                                hipStream_t s, const Win1Desc &w1) {
    const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>((per_rank + STG_WG - 1) / STG_WG,
                                                                          (size_t)num_cu * 8));
    if (world == 1) {
        if (!per_rank) return hipMemsetAsync(out_count, 0, sizeof(uint32_t), s);
        win_mark<<<blocks, STG_WG, 0, s>>>(idx, per_rank, n, win, w1.desc ? w1.dup : nullptr,
                                           w1.desc ? w1.ticket : nullptr);
        const uint32_t nt = (uint32_t)((per_rank + MARK_TILE - 1) / MARK_TILE);
        if (w1.desc) {  // count and emit in one launch (tagged tile counts, look-back)
            constexpr uint32_t wp = 4;  // 1,024-pair tiles (2 / 4 / 16 pairs per thread measured no faster)
            const uint32_t nt1 = (uint32_t)((per_rank + wp * STG_WG - 1) / (wp * STG_WG));
            Win1Args a{idx, val, per_rank, n, nt1, win, w1.desc, w1.ticket, 0ull /* win_mark zeroed it */, w1.tag,
                       out_idx, out_val, out_count, w1.fail, w1.dup, w1.sgd != nullptr,
                       w1.sgd ? *w1.sgd : SgdLaunch{}, w1.adam != nullptr, w1.adam ? *w1.adam : AdamLaunch{}};
            win_emit1t<wp><<<nt1, STG_WG, 0, s>>>(a);
            if (w1.grid_out) *w1.grid_out = nt1;
            return hipGetLastError();
        }
        win_count<<<nt, STG_WG, 0, s>>>(idx, per_rank, n, win, scratch_tiles);
        const uint32_t G = std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)num_cu, nt));
        win_emit1<<<G, STG_WG, 0, s>>>(idx, val, per_rank, n, nt, win, scratch_tiles, out_idx, out_val, out_count);
        return hipGetLastError();
    }
    // rank r's scatter beside rank r+1's election (parity halves of `win`,
    // which holds 2n words for world > 1): world + 1 launches instead of 2 world
    if (per_rank) {
        const uint32_t b2 = (uint32_t)std::max<size_t>(1, std::min<size_t>((2 * per_rank + STG_WG - 1) / STG_WG,
                                                                           (size_t)num_cu * 8));
        for (int r = 0; r <= world; ++r) {
            const bool sc = r >= 1, mk = r < world;
            const size_t ps = (size_t)(r - 1) * per_rank, pm = (size_t)r * per_rank;
            scatter_mark<<<b2, STG_WG, 0, s>>>(sc ? idx + ps : nullptr, sc ? val + ps : nullptr,
                                               win + (size_t)((r - 1) & 1) * n, mk ? idx + pm : nullptr,
                                               win + (size_t)(r & 1) * n, per_rank, n, dense, mark);
        }
    }
    const uint32_t ntiles = (uint32_t)((n + MARK_TILE - 1) / MARK_TILE);
    if (!ntiles) return hipMemsetAsync(out_count, 0, sizeof(uint32_t), s);
    // per-tile counts, their scan, then one workgroup per tile (the old
    // mark_emit walked its tiles one after another: ~90 us at 64 MiB)
    mark_count<<<ntiles, STG_WG, 0, s>>>(mark, n, scratch_tiles);
    mark_scan<<<1, 1024, 0, s>>>(scratch_tiles, ntiles, out_count);
    mark_emit_tile<<<ntiles, STG_WG, 0, s>>>(mark, dense, n, ntiles, (float)world, scratch_tiles, out_idx, out_val);
    return hipGetLastError();
}

hipError_t launch_sgd(const SgdLaunch &a, hipStream_t s) {
    const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((a.grad_len + STG_WG - 1) / STG_WG, 2048));
    sgd_apply<<<blocks, STG_WG, 0, s>>>(a);
    return hipGetLastError();
}

hipError_t launch_adam(const AdamLaunch &a, hipStream_t s) {
    if (!a.amsgrad) {
        const uint32_t blocks = std::max<uint32_t>(1, std::min<uint32_t>((a.grad_len + STG_WG - 1) / STG_WG, 2048));
        adam_apply<<<blocks, STG_WG, 0, s>>>(a);
        return hipGetLastError();
    }
    const uint32_t ntiles = std::max<uint32_t>(1, (a.grad_len + ADAM_TILE - 1) / ADAM_TILE);
    adam_apply_ams<<<ntiles, STG_WG, 0, s>>>(a, a.tag);
    return hipGetLastError();
}

}  // namespace stg
