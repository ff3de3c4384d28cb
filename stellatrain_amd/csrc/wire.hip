// wire.hip -- wire format of the compressed stream (gfx950).
//
// engine/comm_manager.cpp:486-590 packs each (idx, val) stream before it
// leaves for the ZeroMQ ring: u16 indices when tensor_numel < 65536
// (COMM_FLAG_UINT16_IDX, comm_manager.h:24, IDX_COMPRESSION config.h:63) and
// fp16 values under FP16_COMPRESSION (COMM_FLAG_FP16_VAL, compiled out as
// shipped, config.h:64).  The reference casts in 8-wide SIMD blocks while
// i + 8 < length and finishes with a scalar tail, and the halves differ:
//   u32->u16: blocks = signed saturation (_mm_packs_epi32), tail = truncation
//   u16->u32: blocks = sign extension (_mm256_cvtepi16_epi32), tail = zero ext.
//   f32->f16: blocks = IEEE binary16 RNE (_mm256_cvtps_ph(v, 0)); tail =
//             (uint16_t)(int32)trunc(x), fp16_t being uint16_t (comm_manager.h:27)
//   f16->f32: blocks = exact widening; tail = (float) of the uint16 integer
// Both sides reproduce those bytes, so a stream packed here decodes on a
// reference peer exactly as one packed by the reference, and vice versa.
//
// One element per lane, grid-stride: the stream is k pairs (1.3 MB at 64 MiB,
// k = 1 %), so the launch is latency-bound; loads and stores are coalesced
// 4-byte / 2-byte runs per wave.  The fp16 conversion is integer arithmetic so
// NaN payloads and subnormals match the x86 instruction bit for bit.
#include <algorithm>

#include "ws.h"

namespace stg {

namespace {

__device__ __forceinline__ uint32_t f32_to_f16_rne(uint32_t u) {
    const uint32_t sign = (u >> 16) & 0x8000u;
    const uint32_t ex = (u >> 23) & 0xffu;
    uint32_t man = u & 0x7fffffu;
    if (ex == 0xffu) return sign | 0x7c00u | (man ? 0x200u | (man >> 13) : 0u);
    const int e = (int)ex - 112;
    if (e >= 31) return sign | 0x7c00u;
    if (e <= 0) {
        if (e < -10) return sign;
        man |= 0x800000u;
        const uint32_t shift = (uint32_t)(14 - e);
        uint32_t h = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (h & 1u))) ++h;
        return sign | h;
    }
    uint32_t h = ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return sign | h;
}

__device__ __forceinline__ uint32_t f16_to_f32(uint32_t h) {
    const uint32_t sign = (h & 0x8000u) << 16;
    const uint32_t ex = (h >> 10) & 0x1fu;
    uint32_t man = h & 0x3ffu;
    if (ex == 0x1fu) return sign | 0x7f800000u | (man << 13);
    if (ex) return sign | ((ex + 112u) << 23) | (man << 13);
    if (!man) return sign;
    const uint32_t lz = __clz(man) - 21;  // leading zeros within the 11-bit field (man < 0x400)
    man <<= lz;
    return sign | ((113u - lz) << 23) | ((man & 0x3ffu) << 13);
}

__device__ __forceinline__ uint32_t f32_to_u16_trunc(float f) {
    int32_t t = INT32_MIN;  // vcvttss2si r32: invalid -> 0x80000000
    if (f == f && f > -2147483904.0f && f < 2147483648.0f) t = (int32_t)f;
    return (uint32_t)t & 0xffffu;
}

// one element of the encode (shared by the single and the batched launch)
__device__ __forceinline__ void encode_one(const uint32_t *__restrict__ idx, const float *__restrict__ val, size_t i,
                                           size_t simd_end, uint32_t flag, void *__restrict__ idx_out,
                                           void *__restrict__ val_out) {
    const uint32_t x = idx[i];
    if (flag & 1u) {
        const int32_t v = (int32_t)x;
        const uint32_t w = i < simd_end ? (uint32_t)(uint16_t)(int16_t)min(max(v, -32768), 32767) : (x & 0xffffu);
        static_cast<uint16_t *>(idx_out)[i] = (uint16_t)w;
    } else {
        static_cast<uint32_t *>(idx_out)[i] = x;
    }
    const float f = val[i];
    if (flag & 2u)
        static_cast<uint16_t *>(val_out)[i] =
            (uint16_t)(i < simd_end ? f32_to_f16_rne(__float_as_uint(f)) : f32_to_u16_trunc(f));
    else
        static_cast<float *>(val_out)[i] = f;
}

// Batched encode: the launch's workgroups are dealt to the buckets by the
// host-computed first-workgroup offsets (blk0), one element per lane.
__global__ void __launch_bounds__(STG_WG) wire_encode_batch(WireBatch w) {
    uint32_t b = 0;
    while (b + 1 < w.nb && blockIdx.x >= w.b[b + 1].blk0) ++b;
    const WireBucket &d = w.b[b];
    const size_t i = (size_t)(blockIdx.x - d.blk0) * STG_WG + threadIdx.x;
    if (i < d.n) encode_one(d.idx, d.val, i, d.n ? 8 * ((d.n - 1) / 8) : 0, d.flag, d.idx_out, d.val_out);
}

__global__ void __launch_bounds__(STG_WG) wire_encode(const uint32_t *__restrict__ idx, const float *__restrict__ val,
                                                      size_t n, size_t simd_end, uint32_t flag,
                                                      void *__restrict__ idx_out, void *__restrict__ val_out) {
    const size_t stride = (size_t)gridDim.x * STG_WG;
    for (size_t i = (size_t)blockIdx.x * STG_WG + threadIdx.x; i < n; i += stride) {
        encode_one(idx, val, i, simd_end, flag, idx_out, val_out);
    }
}

__global__ void __launch_bounds__(STG_WG) wire_decode(const void *__restrict__ idx_in, const void *__restrict__ val_in,
                                                      size_t n, size_t simd_end, uint32_t flag,
                                                      uint32_t *__restrict__ idx, float *__restrict__ val) {
    const size_t stride = (size_t)gridDim.x * STG_WG;
    for (size_t i = (size_t)blockIdx.x * STG_WG + threadIdx.x; i < n; i += stride) {
        if (flag & 1u) {
            const uint16_t w = static_cast<const uint16_t *>(idx_in)[i];
            idx[i] = i < simd_end ? (uint32_t)(int32_t)(int16_t)w : (uint32_t)w;
        } else {
            idx[i] = static_cast<const uint32_t *>(idx_in)[i];
        }
        if (flag & 2u) {
            const uint16_t h = static_cast<const uint16_t *>(val_in)[i];
            val[i] = i < simd_end ? __uint_as_float(f16_to_f32(h)) : (float)h;
        } else {
            val[i] = static_cast<const float *>(val_in)[i];
        }
    }
}

uint32_t wire_blocks(size_t n, int num_cu) {
    return (uint32_t)std::max<size_t>(1, std::min<size_t>((n + STG_WG - 1) / STG_WG, (size_t)num_cu * 8));
}

size_t simd_end(size_t n) { return n ? 8 * ((n - 1) / 8) : 0; }

}  // namespace

hipError_t launch_wire_encode(const uint32_t *idx, const float *val, size_t n, uint32_t flag, void *idx_out,
                              void *val_out, int num_cu, hipStream_t s) {
    wire_encode<<<wire_blocks(n, num_cu), STG_WG, 0, s>>>(idx, val, n, simd_end(n), flag, idx_out, val_out);
    return hipGetLastError();
}

hipError_t launch_wire_decode(const void *idx_in, const void *val_in, size_t n, uint32_t flag, uint32_t *idx,
                              float *val, int num_cu, hipStream_t s) {
    wire_decode<<<wire_blocks(n, num_cu), STG_WG, 0, s>>>(idx_in, val_in, n, simd_end(n), flag, idx, val);
    return hipGetLastError();
}

hipError_t launch_wire_encode_batch(const WireBatch &w, uint32_t blocks, hipStream_t s) {
    if (!w.nb || !blocks) return hipSuccess;
    wire_encode_batch<<<blocks, STG_WG, 0, s>>>(w);
    return hipGetLastError();
}

}  // namespace stg
