// The reference engine's codec factory and call site, compiled against the
// drop-in header include/stg/compressor.h instead of backend/src/compress/*.h.
//   factory:   engine/core.cpp:110-118 (configure), 185-195 (configure_compression)
//   call site: engine/modules/compress.cpp:141 (MERGE: k = dst capacity, offset 0)
// Usage: shim_factory <method> <in.f32> <k> <out.bin> [calls]
//   reads n floats, runs `calls` compress() calls with key "3@weight" and writes
//   per call: uint64 count, count x uint32 idx, count x float val.
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "stg/compressor.h"

// The engine includes the real engine/threadpool.h; this test only needs the type complete.
class ThreadPool {};

static std::unique_ptr<Compressor> make(const std::string &method, std::unique_ptr<ThreadPool> &pool) {
    std::unique_ptr<Compressor> compressor_;
    if (method == "thresholdv") {
        compressor_ = std::make_unique<ThresholdvCompressor>(pool, true);
    } else if (method == "thresholdv16") {
        compressor_ = std::make_unique<ThresholdvCompressor16>(pool, true);
    } else if (method == "topk") {
        compressor_ = std::make_unique<TopkCompressor>(pool);
    } else {
        throw std::runtime_error(std::string("Unknown compression method ") + method + ".");
    }
    return compressor_;
}

int main(int argc, char **argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s method in.f32 k out.bin [calls]\n", argv[0]);
        return 2;
    }
    std::unique_ptr<ThreadPool> pool;  // never dereferenced, as in the reference codecs
    auto c = make(argv[1], pool);
    FILE *f = fopen(argv[2], "rb");
    if (!f) return 3;
    std::vector<float> src;
    float x;
    while (fread(&x, sizeof x, 1, f) == 1) src.push_back(x);
    fclose(f);
    const uint32_t k = (uint32_t)atoi(argv[3]);
    const int calls = argc > 5 ? atoi(argv[5]) : 1;
    FILE *o = fopen(argv[4], "wb");
    std::vector<uint32_t> idx(k);
    std::vector<float> val(k);
    for (int i = 0; i < calls; ++i) {
        std::fill(idx.begin(), idx.end(), 0u);
        std::fill(val.begin(), val.end(), 0.f);
        auto seg_idx = std::make_pair(idx.data(), (size_t)k);
        auto seg_val = std::make_pair(val.data(), (size_t)k);
        const uint64_t cnt = c->compress("3@weight", std::make_pair((const float *)src.data(), src.size()), k,
                                         seg_idx, seg_val, 0);
        fwrite(&cnt, sizeof cnt, 1, o);
        fwrite(idx.data(), sizeof(uint32_t), cnt, o);
        fwrite(val.data(), sizeof(float), cnt, o);
    }
    fclose(o);
    printf("%s ok\n", c->name().c_str());
    return 0;
}
