// lone_bench.cpp -- the reference's per-task call, timed from C++ (GPU box).
//
// The engine compresses one bucket per ThreadPool task
// (engine/modules/compress.cpp:140-142), from up to 32 workers at once
// (engine/config.h:6-7, core_module_api.cpp:7-24).  Two rows, library
// defaults (no environment knobs), thresholdv16 on 64 MiB buckets, k = 1 %:
//   single   one thread, one stream, back-to-back compress_device calls over
//            16 keys (one distinct bucket each, >= 1 GiB rotating);
//   threads  T threads, each with its own stream and its own 16 keys /
//            buckets, all calling compress_device concurrently; aggregate
//            dense-in GB/s over the slowest thread's span.
// Each row prints one JSON line: device us per call (HIP events), host
// enqueue us per call, GB/s dense-in and the roofline fraction on 4n + 8k.
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 -I include tools/lone_bench.cpp \
//         -L stellatrain_amd -lstg_codec -Wl,-rpath,$PWD/stellatrain_amd -o tools/lone_bench
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "stg/codec.h"

#define HCK(x)                                                                                   \
    do {                                                                                         \
        hipError_t e_ = (x);                                                                     \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)
#define SCK(x)                                                                                   \
    do {                                                                                         \
        if ((x) != STG_OK) { fprintf(stderr, "%s: %s\n", #x, stg_last_error()); exit(1); }       \
    } while (0)

static const size_t N = 16u << 20;       // 64 MiB of fp32
static const uint32_t K = 167772;        // merge_numel(n, 0.99)
static const int KEYS = 16;

struct Lane {  // one caller: a stream, its buckets, keys and outputs
    hipStream_t s;
    std::vector<float *> src;
    std::vector<std::string> key;
    uint32_t *idx, *cnt;
    float *val;
};

static void make_lane(Lane &L, int id) {
    HCK(hipStreamCreateWithFlags(&L.s, hipStreamNonBlocking));
    for (int i = 0; i < KEYS; ++i) {
        float *p;
        HCK(hipMalloc(&p, N * sizeof(float)));
        SCK(stg_synth_fill_device(p, N, 0x5EED0000ull + (100 + 16 * id + i) * 1000ull, 0, 0, L.s));
        L.src.push_back(p);
        L.key.push_back(std::to_string(id) + "." + std::to_string(i) + "@weight");
    }
    HCK(hipMalloc(&L.idx, K * sizeof(uint32_t)));
    HCK(hipMalloc(&L.val, K * sizeof(float)));
    HCK(hipMalloc(&L.cnt, sizeof(uint32_t)));
    HCK(hipStreamSynchronize(L.s));
}

static void call(stg_codec_t h, Lane &L, int i) {
    const int j = i % KEYS;
    SCK(stg_codec_compress_device(h, L.key[j].c_str(), L.src[j], N, K, L.idx, K, L.val, K, 0, L.cnt, L.s));
}

int main(int argc, char **argv) {
    const int threads = argc > 1 ? atoi(argv[1]) : 16;
    const int calls = argc > 2 ? atoi(argv[2]) : 96;
    stg_codec_t h;
    SCK(stg_codec_create("thresholdv16", 0, &h));
    const double alg = 4.0 * N + 8.0 * K;
    // ---- single: one thread, one stream ----
    {
        Lane L;
        make_lane(L, 0);
        for (int i = 0; i < 2 * KEYS; ++i) call(h, L, i);  // first calls + warm-up
        HCK(hipStreamSynchronize(L.s));
        hipEvent_t e0, e1;
        HCK(hipEventCreate(&e0));
        HCK(hipEventCreate(&e1));
        HCK(hipEventRecord(e0, L.s));
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < calls; ++i) call(h, L, i);
        const double host_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        HCK(hipEventRecord(e1, L.s));
        HCK(hipEventSynchronize(e1));
        float ms = 0;
        HCK(hipEventElapsedTime(&ms, e0, e1));
        SCK(stg_codec_check(h));
        const double us = ms * 1e3 / calls;
        printf("{\"config\": \"thresholdv16 single-bucket 64 MiB k=%u, C++ caller, library defaults\", \"us_per_call\": "
               "%.2f, \"host_enqueue_us_per_call\": %.2f, \"GBps_dense_in\": %.1f, \"frac_hbm_peak\": %.4f, \"calls\": %d}\n",
               K, us, host_us / calls, 4.0 * N / us / 1e3, alg / us / 1e3 / 8000.0, calls);
        fflush(stdout);
    }
    // ---- threads: T callers on their own streams ----
    if (threads > 0) {
        std::vector<Lane> lanes(threads);
        for (int t = 0; t < threads; ++t) make_lane(lanes[t], t + 1);
        for (int t = 0; t < threads; ++t)
            for (int i = 0; i < 2 * KEYS; ++i) call(h, lanes[t], i);
        HCK(hipDeviceSynchronize());
        std::atomic<int> ready{0};
        std::atomic<bool> go{false};
        std::vector<double> span(threads);
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t] {
                HCK(hipSetDevice(0));
                ready++;
                while (!go.load()) std::this_thread::yield();
                const auto t0 = std::chrono::steady_clock::now();
                for (int i = 0; i < calls; ++i) call(h, lanes[t], i);
                HCK(hipStreamSynchronize(lanes[t].s));
                span[t] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
            });
        while (ready.load() < threads) std::this_thread::yield();
        const auto w0 = std::chrono::steady_clock::now();
        go = true;
        for (auto &x : th) x.join();
        const double wall = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - w0).count();
        SCK(stg_codec_check(h));
        const double bytes = 4.0 * N * threads * calls;
        printf("{\"config\": \"thresholdv16 64 MiB k=%u: %d host threads x lone compress_device on their own streams, "
               "library defaults\", \"threads\": %d, \"calls_per_thread\": %d, \"wall_us\": %.1f, \"GBps_dense_in\": %.1f, "
               "\"alg_GBps\": %.1f, \"frac_hbm_peak\": %.4f, \"us_per_bucket\": %.2f}\n",
               K, threads, threads, calls, wall, bytes / wall / 1e3, alg * threads * calls / wall / 1e3,
               alg * threads * calls / wall / 1e3 / 8000.0, wall / (threads * calls));
    }
    stg_codec_destroy(h);
    return 0;
}
