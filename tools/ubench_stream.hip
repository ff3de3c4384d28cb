// ubench_stream.hip -- streaming-read calibration for the codec's scan pass.
// Reads 64 MiB fp32 buckets rotating through 1 GiB, reducing each float4 to a
// flag (like the codec), under different launch shapes.  Prints one line per
// configuration: microseconds per bucket and GB/s (median of 5 x 64 buckets).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_stream.hip -o /tmp/ubench_stream
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdio>
#include <vector>

typedef float f4v __attribute__((ext_vector_type(4)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int WG, int U, bool NT>
__global__ void __launch_bounds__(WG) k_static(const float4 *__restrict__ src, size_t n4, unsigned *out) {
    const size_t per = (n4 + gridDim.x - 1) / gridDim.x;
    const size_t b0 = blockIdx.x * per, b1 = min(n4, b0 + per);
    unsigned c = 0;
    for (size_t i = b0 + threadIdx.x; i < b1; i += (size_t)WG * U) {
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = i + (size_t)u * WG;
            const size_t jc = j < b1 ? j : b0;
            if (NT) {
                const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(src + jc));
                v[u] = make_float4(t.x, t.y, t.z, t.w);
            } else {
                v[u] = src[jc];
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) c += (v[u].x + v[u].y + v[u].z + v[u].w) > 1e30f;
    }
    if (c == 12345) out[0] = c;
}

template <int WG, int U>
__global__ void __launch_bounds__(WG) k_chunks(const float4 *__restrict__ src, size_t n4, unsigned *ctr,
                                               unsigned *out) {
    // dynamic chunks of WG*U float4 claimed from an atomic counter
    __shared__ unsigned s_c;
    const size_t chunk = (size_t)WG * U;
    const unsigned nch = (unsigned)((n4 + chunk - 1) / chunk);
    unsigned c = 0;
    for (;;) {
        if (threadIdx.x == 0) s_c = atomicAdd(ctr, 1u);
        __syncthreads();
        const unsigned ch = s_c;
        __syncthreads();
        if (ch >= nch) break;
        float4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const size_t j = (size_t)ch * chunk + (size_t)u * WG + threadIdx.x;
            v[u] = src[j < n4 ? j : 0];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) c += (v[u].x + v[u].y + v[u].z + v[u].w) > 1e30f;
    }
    if (c == 12345) out[0] = c;
}

template <int WG, bool NT = false>
__global__ void __launch_bounds__(WG) k_onepass(const float4 *__restrict__ src, size_t n4, unsigned *out) {
    // one float4 x 8 per thread, grid = n4 / (WG*8): the v1 scan shape
    const size_t i = (size_t)blockIdx.x * WG * 8 + threadIdx.x;
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const size_t j = min(i + (size_t)u * WG, n4 - 1);
        if (NT) {
            const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v *>(src + j));
            v[u] = make_float4(t.x, t.y, t.z, t.w);
        } else {
            v[u] = src[j];
        }
    }
    unsigned c = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) c += (v[u].x + v[u].y + v[u].z + v[u].w) > 1e30f;
    if (c == (unsigned)n4 + 7u) out[0] = c;  // (not provably false: the loads stay)
}

int main(int argc, char **argv) {
    const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 64;  // bucket size (MiB), rotating through >= 1 GiB
    const size_t n = mib << 18, n4 = n / 4;
    const int NB = (int)std::max<size_t>(2, 1024 / mib);
    std::vector<float *> bufs(NB);
    for (auto &b : bufs) { CK(hipMalloc(&b, n * 4)); CK(hipMemset(b, 0, n * 4)); }
    unsigned *out, *ctr;
    CK(hipMalloc(&out, 64));
    CK(hipMalloc(&ctr, 4 * 4096));
    CK(hipMemset(ctr, 0, 4 * 4096));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        std::vector<float> ms;
        for (int rep = 0; rep < 6; ++rep) {
            CK(hipMemset(ctr, 0, 4 * 4096));
            CK(hipEventRecord(e0));
            for (int i = 0; i < 64; ++i) launch(i, bufs[i % NB]);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (rep) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        const double us = ms[ms.size() / 2] * 1e3 / 64;
        printf("%-34s %8.2f us  %7.1f GB/s\n", name, us, n * 4.0 / (us * 1e-6) / 1e9);
        return 0;
    };
    char nm[128];
    run("onepass WG256 U8 (v1 scan)", [&](int, float *b) {
        k_onepass<256><<<(unsigned)(n4 / 2048), 256>>>((const float4 *)b, n4, out);
    });
    run("onepass WG256 U8 nt", [&](int, float *b) {
        k_onepass<256, true><<<(unsigned)(n4 / 2048), 256>>>((const float4 *)b, n4, out);
    });
#define STATIC(WG, U, NT, PER)                                                                             \
    snprintf(nm, sizeof nm, "static WG%d U%d nt%d x%d/CU", WG, U, (int)NT, PER);                          \
    run(nm, [&](int, float *b) { k_static<WG, U, NT><<<ncu * PER, WG>>>((const float4 *)b, n4, out); });
    STATIC(1024, 16, false, 1)
    STATIC(1024, 8, false, 1)
    STATIC(1024, 8, false, 2)
    STATIC(512, 16, false, 2)
    STATIC(512, 8, false, 4)
    STATIC(256, 16, false, 4)
    STATIC(256, 8, false, 8)
    STATIC(256, 16, false, 8)
    STATIC(1024, 16, true, 1)
    STATIC(256, 8, true, 8)
#define CHUNKS(WG, U, PER)                                                                                 \
    snprintf(nm, sizeof nm, "chunks WG%d U%d x%d/CU", WG, U, PER);                                      \
    run(nm, [&](int i, float *b) { k_chunks<WG, U><<<ncu * PER, WG>>>((const float4 *)b, n4, ctr + (i % 64), out); });
    CHUNKS(1024, 16, 1)
    CHUNKS(1024, 8, 2)
    CHUNKS(256, 16, 4)
    CHUNKS(256, 8, 8)
    return 0;
}
