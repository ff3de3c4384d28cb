// wire_dev.h -- the wire form of one (idx, val) pair, shared by the wire
// encode (wire.hip) and the thresholdv16 emission that writes it directly
// (tv16*.hip: stg_codec_compress_wire_device).  gfx950 only.
//
// Pair i of a stream of numel pairs is packed by its position
// (comm_manager.cpp:486-590): i < wend = 8 * ((numel - 1) / 8) is the
// reference's SIMD-block part, the rest its scalar tail (see wire.hip).
#pragma once

#include <stdint.h>

// 0: the emission ignores the wire flag (an A/B build of the codegen cost)
#ifndef STG_WIRE_EMIT
#define STG_WIRE_EMIT 1
#endif

namespace stg {

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

// u16 index: blocks saturate as signed 16-bit (_mm_packs_epi32), the tail truncates
__device__ __forceinline__ uint32_t wire_idx16(uint32_t x, size_t i, size_t wend) {
    return i < wend ? (uint32_t)(uint16_t)(int16_t)min(max((int32_t)x, -32768), 32767) : (x & 0xffffu);
}
// fp16 value: blocks round to nearest even (_mm256_cvtps_ph), the tail truncates to an integer
__device__ __forceinline__ uint32_t wire_val16(float f, size_t i, size_t wend) {
    return i < wend ? f32_to_f16_rne(__float_as_uint(f)) : f32_to_u16_trunc(f);
}

// Pair `o` of the stream in the form `flag` selects (STG_WIRE_U16_IDX = 1,
// STG_WIRE_F16_VAL = 2; 0: the codec's own u32 / f32).
__device__ __forceinline__ void wire_put(uint32_t *idx, float *val, uint32_t flag, uint32_t wend, uint32_t o,
                                         uint32_t ix, float v) {
    if (flag & 1u) reinterpret_cast<uint16_t *>(idx)[o] = (uint16_t)wire_idx16(ix, o, wend);
    else idx[o] = ix;
    if (flag & 2u) reinterpret_cast<uint16_t *>(val)[o] = (uint16_t)wire_val16(v, o, wend);
    else val[o] = v;
}

// Pairs o..o+3 (o % 4 == 0, so all four sit on one side of wend, a multiple
// of 8): bi..bi+3 with values x, as 8-byte stores of the 16-bit forms.
__device__ __forceinline__ void wire_put4(uint32_t *idx, float *val, uint32_t flag, uint32_t wend, uint32_t o,
                                          uint32_t bi, float4 x) {
    if (flag & 1u) {
        const uint32_t a = wire_idx16(bi, o, wend), b = wire_idx16(bi + 1, o, wend);
        const uint32_t c = wire_idx16(bi + 2, o, wend), e = wire_idx16(bi + 3, o, wend);
        *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(idx) + o) = make_uint2(a | b << 16, c | e << 16);
    } else {
        *reinterpret_cast<uint4 *>(idx + o) = make_uint4(bi, bi + 1, bi + 2, bi + 3);
    }
    if (flag & 2u) {
        const uint32_t a = wire_val16(x.x, o, wend), b = wire_val16(x.y, o, wend);
        const uint32_t c = wire_val16(x.z, o, wend), e = wire_val16(x.w, o, wend);
        *reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(val) + o) = make_uint2(a | b << 16, c | e << 16);
    } else {
        *reinterpret_cast<float4 *>(val + o) = x;
    }
}

// One emitted pair through a bucket descriptor (fields idx, val, wflag,
// wend): W = the stream takes its wire form (the caller has tested d.wflag).
template <bool W, typename D>
__device__ __forceinline__ void put_pair_w(const D &d, uint32_t o, uint32_t ix, float v) {
    if (W) {
        wire_put(d.idx, d.val, d.wflag, d.wend, o, ix, v);
    } else {
        d.val[o] = v;
        d.idx[o] = ix;
    }
}
// Four pairs (16-byte aligned buffers, o % 4 == 0).
template <bool W, typename D>
__device__ __forceinline__ void put_pair4_w(const D &d, uint32_t o, uint32_t bi, float4 x) {
    if (W) {
        wire_put4(d.idx, d.val, d.wflag, d.wend, o, bi, x);
    } else {
        *reinterpret_cast<float4 *>(d.val + o) = x;
        *reinterpret_cast<uint4 *>(d.idx + o) = make_uint4(bi, bi + 1, bi + 2, bi + 3);
    }
}
// The same with the flag tested here (emission sites off the fill's hot loops).
template <typename D>
__device__ __forceinline__ void put_pair(const D &d, uint32_t o, uint32_t ix, float v) {
    if (STG_WIRE_EMIT && d.wflag) put_pair_w<true>(d, o, ix, v);
    else put_pair_w<false>(d, o, ix, v);
}
template <typename D>
__device__ __forceinline__ void put_pair4(const D &d, uint32_t o, uint32_t bi, float4 x) {
    if (STG_WIRE_EMIT && d.wflag) put_pair4_w<true>(d, o, bi, x);
    else put_pair4_w<false>(d, o, bi, x);
}

}  // namespace stg
