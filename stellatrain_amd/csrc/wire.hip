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
// The per-element casts live in wire_dev.h, shared with the thresholdv16
// emission that writes the wire form directly.  One element per lane,
// grid-stride: the stream is k pairs (1.3 MB at 64 MiB, k = 1 %), so the launch is latency-bound; loads and stores are coalesced
// 4-byte / 2-byte runs per wave.  The fp16 conversion is integer arithmetic so
// NaN payloads and subnormals match the x86 instruction bit for bit.
#include <algorithm>

#include "ws.h"
#include "wire_dev.h"

namespace stg {

namespace {

// one element of the encode (shared by the single and the batched launch)
__device__ __forceinline__ void encode_one(const uint32_t *__restrict__ idx, const float *__restrict__ val, size_t i,
                                           size_t simd_end, uint32_t flag, void *__restrict__ idx_out,
                                           void *__restrict__ val_out) {
    const uint32_t x = idx[i];
    if (flag & 1u) static_cast<uint16_t *>(idx_out)[i] = (uint16_t)wire_idx16(x, i, simd_end);
    else static_cast<uint32_t *>(idx_out)[i] = x;
    const float f = val[i];
    if (flag & 2u) static_cast<uint16_t *>(val_out)[i] = (uint16_t)wire_val16(f, i, simd_end);
    else static_cast<float *>(val_out)[i] = f;
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
