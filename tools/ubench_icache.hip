// ubench_icache.hip -- does a cold instruction stream cost microseconds?
// Kernel `straight` runs ~N_OPS dependent-free VALU ops as straight-line code
// (one 512-thread workgroup); it is timed (HIP events, mean of 200 launches)
// back to back, and each time right after `stream` reads 64 MiB (which sweeps
// the L2s).  hipcc -O2 --offload-arch=gfx950 tools/ubench_icache.hip -o tools/ubench_icache
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
#define OPS R8(R8(R8(asm volatile("v_add_f32 %0, %0, %1\n\tv_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));)))

__global__ void __launch_bounds__(512) straight(float *out, float b) {
    float a = threadIdx.x;
    OPS OPS OPS OPS OPS OPS OPS OPS  // 8 x 512 x 2 = 8192 instructions (~64 KB)
    if (a == 1234.5f) out[threadIdx.x] = a;
}
__global__ void __launch_bounds__(512) short_k(float *out, float b) {
    float a = threadIdx.x;
    for (int i = 0; i < 4096; ++i) asm volatile("v_add_f32 %0, %0, %1\n\tv_mul_f32 %0, %0, %1" : "+v"(a) : "v"(b));
    if (a == 1234.5f) out[threadIdx.x] = a;
}
__global__ void stream(const float4 *p, size_t n4, float *out) {
    float s = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = __builtin_nontemporal_load(&p[i].x) == 0 ? p[i] : p[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1234.5f) out[0] = s;
}

int main() {
    const size_t n4 = (64u << 20) / 16;
    float4 *buf; float *out;
    hipMalloc(&buf, n4 * 16); hipMalloc(&out, 4096);
    hipMemset(buf, 0, n4 * 16);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto time = [&](const char *name, bool cold, bool longk) {
        float tot = 0;
        for (int i = 0; i < 200; ++i) {
            if (cold) stream<<<2048, 256>>>(buf, n4, out);
            hipEventRecord(e0);
            if (longk) straight<<<1, 512>>>(out, 1.0f); else short_k<<<1, 512>>>(out, 1.0f);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            if (i >= 20) tot += ms;
        }
        printf("{\"kernel\": \"%s\", \"after_64MiB_stream\": %s, \"us\": %.2f}\n", name, cold ? "true" : "false", tot * 1e3 / 180);
    };
    time("straight 8192 insts", false, true);
    time("straight 8192 insts", true, true);
    time("loop 8192 insts", false, false);
    time("loop 8192 insts", true, false);
    return 0;
}
