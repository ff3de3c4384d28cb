// synth.hip -- synthetic gradient buckets from an integer-only generator.
//
// Bit-identical to oracle/stg_oracle.cpp:orc_synth_fill and
// stellatrain_amd/synth.py (std::normal_distribution changes with
// -O level, so the fixtures use splitmix64 + Irwin-Hall(4) of 24-bit uniforms).
#include "ws.h"

namespace stg {

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__global__ void __launch_bounds__(STG_WG) synth_fill(float *__restrict__ dst, size_t n, uint64_t seed, int dist,
                                                     uint32_t param) {
    const double scale = 1e-3 / 16777216.0;
    const size_t stride = (size_t)gridDim.x * STG_WG;
    for (size_t i = (size_t)blockIdx.x * STG_WG + threadIdx.x; i < n; i += stride) {
        const uint64_t base = seed * 0x100000001B3ull + (uint64_t)i * 4u;
        const uint64_t r0 = splitmix64(base + 0), r1 = splitmix64(base + 1);
        const int64_t v = (int64_t)(r0 & 0xFFFFFF) + (int64_t)((r0 >> 24) & 0xFFFFFF) + (int64_t)(r1 & 0xFFFFFF) +
                          (int64_t)((r1 >> 24) & 0xFFFFFF) - (int64_t{1} << 25);
        double x = (double)v * scale;
        if (dist == 1) {
            const uint32_t e = (uint32_t)((r1 >> 48) % 9u);
            x = x * (1.0 / (double)(1u << e));  // exact power-of-two scaling
        } else if (dist == 2) {
            const uint32_t z = (uint32_t)((r0 >> 48) % 10000u);
            if (z < param) x = 0.0;
        }
        dst[i] = (float)x;
    }
}

}  // namespace

hipError_t launch_synth(float *dst, size_t n, uint64_t seed, int dist, uint32_t param, hipStream_t s) {
    const size_t blocks = std::min<size_t>((n + STG_WG - 1) / STG_WG, 16384);
    synth_fill<<<(uint32_t)std::max<size_t>(blocks, 1), STG_WG, 0, s>>>(dst, n, seed, dist, param);
    return hipGetLastError();
}

}  // namespace stg
