// ubench_idle.hip -- what an idle follow-on launch costs behind a streaming
// kernel: a gated kernel that reads one flag and returns, with and without a
// private (scratch) segment in its descriptor.  Prints us per (stream + idle)
// pair against the stream alone (median of 7 x 200 pairs).
//   hipcc -O3 --offload-arch=gfx950 tools/ubench_idle.hip -o tools/ubench_idle
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void __launch_bounds__(256) k_stream(const float4 *__restrict__ src, size_t n4, unsigned *out) {
    const size_t i = (size_t)blockIdx.x * 2048 + threadIdx.x;
    float4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[min(i + (size_t)u * 256, n4 - 1)];
    unsigned c = 0;
#pragma unroll
    for (int u = 0; u < 8; ++u) c += (v[u].x + v[u].y + v[u].z + v[u].w) > 1e30f;
    if (c == (unsigned)n4 + 7u) out[0] = c;
}

// gated: every thread reads the flag word; the rest never runs (flag != 1)
template <int SCRATCH>
__global__ void __launch_bounds__(512) k_idle(const unsigned *flag, unsigned *out, unsigned sel) {
    if (__syncthreads_or(flag[threadIdx.x & 63] != 1u)) return;
    if constexpr (SCRATCH > 0) {
        volatile float priv[SCRATCH];
        for (unsigned i = 0; i < (unsigned)SCRATCH; ++i) priv[(i * 7 + sel) % SCRATCH] = (float)i;
        out[threadIdx.x] = (unsigned)priv[sel % SCRATCH];
    } else {
        out[threadIdx.x] = sel;
    }
}

struct Big {  // a 1.5 KiB argument block, like the fill launch's
    const unsigned *flag;
    unsigned *out;
    unsigned pad[376];
};
__global__ void __launch_bounds__(512) k_idle_big(Big b) {
    if (__syncthreads_or(b.flag[threadIdx.x & 63] != 1u)) return;
    b.out[threadIdx.x] = b.pad[threadIdx.x % 376];
}

int main() {
    const size_t n = 16u << 20, n4 = n / 4;
    const int NB = 16;
    std::vector<float *> bufs(NB);
    for (auto &b : bufs) { CK(hipMalloc(&b, n * 4)); CK(hipMemset(b, 0, n * 4)); }
    unsigned *out, *flag;
    CK(hipMalloc(&out, 4096));
    CK(hipMalloc(&flag, 4096));
    CK(hipMemset(flag, 0, 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char *name, auto launch) {
        std::vector<float> ms;
        for (int rep = 0; rep < 8; ++rep) {
            CK(hipEventRecord(e0));
            for (int i = 0; i < 200; ++i) launch(bufs[i % NB]);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float t;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (rep) ms.push_back(t);
        }
        std::sort(ms.begin(), ms.end());
        printf("%-44s %8.2f us per iteration\n", name, ms[ms.size() / 2] * 1e3 / 200);
        return 0;
    };
    const unsigned G = (unsigned)(n4 / 2048);
    run("stream alone (64 MiB)", [&](float *b) { k_stream<<<G, 256>>>((const float4 *)b, n4, out); });
    run("stream + idle 72 WG, no scratch", [&](float *b) {
        k_stream<<<G, 256>>>((const float4 *)b, n4, out);
        k_idle<0><<<72, 512>>>(flag, out, 3);
    });
    run("stream + idle 72 WG, 580 B scratch / lane", [&](float *b) {
        k_stream<<<G, 256>>>((const float4 *)b, n4, out);
        k_idle<145><<<72, 512>>>(flag, out, 3);
    });
    run("stream + idle 512 WG, 136 B scratch / lane", [&](float *b) {
        k_stream<<<G, 256>>>((const float4 *)b, n4, out);
        k_idle<34><<<512, 512>>>(flag, out, 3);
    });
    run("stream + idle 512 WG, no scratch", [&](float *b) {
        k_stream<<<G, 256>>>((const float4 *)b, n4, out);
        k_idle<0><<<512, 512>>>(flag, out, 3);
    });
    Big big{};
    big.flag = flag;
    big.out = out;
    run("stream + idle 72 WG, 1.5 KiB argument block", [&](float *b) {
        k_stream<<<G, 256>>>((const float4 *)b, n4, out);
        k_idle_big<<<72, 512>>>(big);
    });
    return 0;
}
