// The reference's threading contract, exercised on one codec handle.
//
// The engine calls compressor()->compress() from up to 32 ThreadPool workers
// at once, each on its own key (engine/config.h:6-7, engine/core_module_api.cpp:
// 7-24, engine/modules/compress.cpp:140-142); thresholdv16 guards its
// per-name threshold maps with a mutex (compress/thresholdv16.cpp:84,256).
// Here T std::threads share ONE handle (include/stg/compressor.h) and each
// runs `calls` AIMD iterations on two keys of its own:
//   "<t>@host"  through compress()        (host memory; the handle's per-thread
//                                          stream, stg_codec_compress_host)
//   "<t>@dev"   through compress_device() (device memory, on a HIP stream this
//                                          thread created: the reference idiom of
//                                          per-worker streams, d2h_copy.h:10-17)
// interleaved call by call, all threads released together.  Inputs come from
// the integer-only generator (stg_synth_fill_device, bit-identical to the
// oracle's): bucket t, call c has seed 1000 t + c (host key) and
// 1000 t + 500 + c (device key), n_t = n + 5 (t % 4) floats, k_t = n_t / 100.
// Every call's (count, idx, val) stream and the key's threshold / increment
// bits after it go to <out>.<t>; tests/test_gpu_concurrency.py replays each
// key's sequence through the oracle and compares everything bit for bit.
//
// Usage: concurrency <method> <threads> <calls> <n> <out-prefix>
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "stg/compressor.h"

class ThreadPool {};

#define HCK(x)                                                                           \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) throw std::runtime_error(std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)
#define SCK(x)                                                                           \
    do {                                                                                 \
        if ((x) != STG_OK) throw std::runtime_error(std::string(#x ": ") + stg_last_error()); \
    } while (0)

static std::unique_ptr<Compressor> make(const std::string &method, std::unique_ptr<ThreadPool> &pool) {
    if (method == "thresholdv16") return std::make_unique<ThresholdvCompressor16>(pool, true);
    if (method == "thresholdv") return std::make_unique<ThresholdvCompressor>(pool, true);
    if (method == "topk") return std::make_unique<TopkCompressor>(pool);
    throw std::runtime_error("Unknown compression method " + method + ".");
}

struct Rec {
    FILE *f;
    void put(const void *p, size_t bytes) { fwrite(p, 1, bytes, f); }
};

int main(int argc, char **argv) {
    if (argc < 6) {
        fprintf(stderr, "usage: %s method threads calls n out-prefix\n", argv[0]);
        return 2;
    }
    const std::string method = argv[1];
    const int T = atoi(argv[2]), calls = atoi(argv[3]);
    const size_t n0 = strtoull(argv[4], nullptr, 10);
    const std::string out = argv[5];
    const bool stateful = method != "topk";  // Top-k keeps no per-key state
    std::unique_ptr<ThreadPool> pool;
    auto comp = make(method, pool);
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<std::string> errs(T);
    auto worker = [&](int t) {
        try {
            HCK(hipSetDevice(0));
            const size_t n = n0 + 5 * (t % 4);
            const uint32_t k = (uint32_t)(n / 100);
            hipStream_t s;
            HCK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
            float *d_src = nullptr, *d_val = nullptr;
            uint32_t *d_idx = nullptr, *d_cnt = nullptr;
            HCK(hipMalloc(&d_src, n * sizeof(float)));
            HCK(hipMalloc(&d_val, k * sizeof(float)));
            HCK(hipMalloc(&d_idx, k * sizeof(uint32_t)));
            HCK(hipMalloc(&d_cnt, sizeof(uint32_t)));
            float *h_src = nullptr;  // pinned, like the reference's registered shm
            HCK(hipHostMalloc(&h_src, n * sizeof(float), 0));
            std::vector<uint32_t> idx(k);
            std::vector<float> val(k);
            Rec r{fopen((out + "." + std::to_string(t)).c_str(), "wb")};
            if (!r.f) throw std::runtime_error("cannot open output");
            const std::string kh = std::to_string(t) + "@host", kd = std::to_string(t) + "@dev";
            ready.fetch_add(1);
            while (!go.load()) std::this_thread::yield();
            for (int c = 0; c < calls; ++c) {
                // host path: the bucket generated on the device, copied to pinned host memory
                SCK(stg_synth_fill_device(d_src, n, 1000ull * t + c, 0, 0, s));
                HCK(hipMemcpyAsync(h_src, d_src, n * sizeof(float), hipMemcpyDeviceToHost, s));
                HCK(hipStreamSynchronize(s));
                std::fill(idx.begin(), idx.end(), 0u);
                std::fill(val.begin(), val.end(), 0.f);
                const uint64_t ch = comp->compress(kh, std::make_pair((const float *)h_src, n), k,
                                                   std::make_pair(idx.data(), (size_t)k),
                                                   std::make_pair(val.data(), (size_t)k), 0);
                float th = 0, ih = 0;
                if (stateful) SCK(stg_codec_get_state(comp->handle(), kh.c_str(), h_src, &th, &ih, nullptr));
                uint32_t tag = 0;
                r.put(&tag, 4);
                r.put(&ch, 8);
                r.put(idx.data(), 4 * ch);
                r.put(val.data(), 4 * ch);
                r.put(&th, 4);
                r.put(&ih, 4);
                // device path on this thread's stream
                SCK(stg_synth_fill_device(d_src, n, 1000ull * t + 500 + c, 0, 0, s));
                HCK(hipMemsetAsync(d_idx, 0, k * sizeof(uint32_t), s));
                HCK(hipMemsetAsync(d_val, 0, k * sizeof(float), s));
                comp->compress_device(kd, std::make_pair((const float *)d_src, n), k, std::make_pair(d_idx, (size_t)k),
                                      std::make_pair(d_val, (size_t)k), d_cnt, s, 0);
                uint32_t cd = 0;
                HCK(hipMemcpyAsync(&cd, d_cnt, 4, hipMemcpyDeviceToHost, s));
                HCK(hipMemcpyAsync(idx.data(), d_idx, k * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
                HCK(hipMemcpyAsync(val.data(), d_val, k * sizeof(float), hipMemcpyDeviceToHost, s));
                HCK(hipStreamSynchronize(s));
                if (cd > k) throw std::runtime_error("device count past capacity (poisoned?)");
                float td = 0, id = 0;
                if (stateful) SCK(stg_codec_get_state(comp->handle(), kd.c_str(), d_src, &td, &id, s));
                const uint64_t cd64 = cd;
                tag = 1;
                r.put(&tag, 4);
                r.put(&cd64, 8);
                r.put(idx.data(), 4 * cd);
                r.put(val.data(), 4 * cd);
                r.put(&td, 4);
                r.put(&id, 4);
            }
            fclose(r.f);
            HCK(hipStreamSynchronize(s));
            HCK(hipFree(d_src));
            HCK(hipFree(d_val));
            HCK(hipFree(d_idx));
            HCK(hipFree(d_cnt));
            HCK(hipHostFree(h_src));
            HCK(hipStreamDestroy(s));
        } catch (const std::exception &e) {
            errs[t] = e.what();
            ready.fetch_add(1);
        }
    };
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) th.emplace_back(worker, t);
    while (ready.load() < T) std::this_thread::yield();
    go.store(true);
    for (auto &x : th) x.join();
    int bad = 0;
    for (int t = 0; t < T; ++t)
        if (!errs[t].empty()) {
            fprintf(stderr, "thread %d: %s\n", t, errs[t].c_str());
            ++bad;
        }
    if (stg_codec_check(comp->handle()) != STG_OK) {
        fprintf(stderr, "device failure: %s\n", stg_last_error());
        ++bad;
    }
    if (bad) return 1;
    printf("%s: %d threads x %d calls ok\n", comp->name().c_str(), T, calls);
    return 0;
}
