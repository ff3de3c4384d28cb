// gather.hip -- intra-node gather-add before the codec (gfx950).
//
// ModuleCpuGather::run (engine/modules/cpu_gather.cpp:59-87): local rank r of
// N owns the slice [len*r/N, len*(r+1)/N) of grad[0] and adds into it, in
// order, the residual and grad[1] .. grad[N-1] with add_arrays
// (misc/array_util.h:12-54, a plain per-element dst += src).  Here the N - 1
// sources are device pointers -- this GPU's buffers or peers' over xGMI (P2P
// enabled or IPC-mapped) -- and the whole chain is one pass: each element is
// read once from every source, summed in the reference's order in a register
// and stored once, instead of N read-modify-write passes over dst.
//
// Bound: HBM (or xGMI for peer sources); algorithmic bytes per element
// 4 (dst) + 4 (residual) + 4 (N - 1) + 4 (store).  float4 lanes when every
// slice pointer shares one 16-byte phase (the head elements go scalar),
// nontemporal loads of the sources.
#include <algorithm>

#include "ws.h"

namespace stg {

namespace {

typedef float f4v __attribute__((ext_vector_type(4)));

// MAXS >= nsrc: every source's float4 is loaded before any is added (a
// runtime-length loop of load-then-add waited for each load in turn), then
// the sum runs in the reference's order: dst, residual, grad[1], ...
template <uint32_t MAXS>
__global__ void __launch_bounds__(STG_WG) gather_add_vec(GatherArgs a, size_t v0, size_t nv) {
    const size_t stride = (size_t)gridDim.x * STG_WG;
    for (size_t i = (size_t)blockIdx.x * STG_WG + threadIdx.x; i < nv; i += stride) {
        const size_t e = v0 + 4 * i;
        f4v x[MAXS];
        f4v acc = *reinterpret_cast<const f4v *>(a.dst + e);
        const f4v r = a.resid ? __builtin_nontemporal_load(reinterpret_cast<const f4v *>(a.resid + e)) : f4v{0, 0, 0, 0};
#pragma unroll
        for (uint32_t s = 1; s < MAXS; ++s)
            if (s < a.nsrc) x[s] = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(a.src[s] + e));
        if (a.resid) acc += r;
#pragma unroll
        for (uint32_t s = 1; s < MAXS; ++s)
            if (s < a.nsrc) acc += x[s];
        *reinterpret_cast<f4v *>(a.dst + e) = acc;
    }
}

__global__ void __launch_bounds__(STG_WG) gather_add_scalar(GatherArgs a, size_t b0, size_t b1) {
    const size_t stride = (size_t)gridDim.x * STG_WG;
    for (size_t e = b0 + (size_t)blockIdx.x * STG_WG + threadIdx.x; e < b1; e += stride) {
        float acc = a.dst[e];
        if (a.resid) acc += a.resid[e];
        for (uint32_t s = 1; s < a.nsrc; ++s) acc += a.src[s][e];
        a.dst[e] = acc;
    }
}

}  // namespace

hipError_t launch_gather_add(const GatherArgs &a, size_t start, size_t end, int num_cu, hipStream_t s) {
    if (end <= start) return hipSuccess;
    // the 16-byte phase of the slice start must agree across every pointer
    auto phase = [&](const float *p) { return (reinterpret_cast<uintptr_t>(p + start) & 15u); };
    const uintptr_t ph = phase(a.dst);
    bool vec = (ph & 3u) == 0;
    if (a.resid) vec &= phase(a.resid) == ph;
    for (uint32_t i = 1; i < a.nsrc; ++i) vec &= phase(a.src[i]) == ph;
    size_t head = vec ? std::min<size_t>(end - start, ((16u - ph) & 15u) / 4u) : end - start;
    const size_t v0 = start + head, nv = vec ? (end - v0) / 4 : 0, vt = v0 + 4 * nv;
    const uint32_t cap = (uint32_t)num_cu * 8;
    if (nv) {
        const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>((nv + STG_WG - 1) / STG_WG, cap));
        if (a.nsrc <= 4) gather_add_vec<4><<<blocks, STG_WG, 0, s>>>(a, v0, nv);
        else if (a.nsrc <= 8) gather_add_vec<8><<<blocks, STG_WG, 0, s>>>(a, v0, nv);
        else gather_add_vec<GATHER_MAX><<<blocks, STG_WG, 0, s>>>(a, v0, nv);
    }
    if (head) {
        const uint32_t blocks = (uint32_t)std::max<size_t>(1, std::min<size_t>((head + STG_WG - 1) / STG_WG, cap));
        gather_add_scalar<<<blocks, STG_WG, 0, s>>>(a, start, start + head);
    }
    if (vec && end > vt) gather_add_scalar<<<1, STG_WG, 0, s>>>(a, vt, end);
    return hipGetLastError();
}

}  // namespace stg
