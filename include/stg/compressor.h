/*
 * stg/compressor.h -- header-only C++ drop-in for backend/src/compress.
 *
 * Same class names, constructors and virtual compress() as the reference
 *   compressor.h:12-31   class Compressor (Segment / ConstSegment, name(), compress)
 *   thresholdv16.h:33-35 ThresholdvCompressor16(std::unique_ptr<ThreadPool>&, bool multicore = true)
 *   thresholdv.h:24-26   ThresholdvCompressor(std::unique_ptr<ThreadPool>&, bool multicore = true)
 *   topk.h:28-30         TopkCompressor(std::unique_ptr<ThreadPool>&)
 * so the engine's factory (engine/core.cpp:110-118, 185-195) and its call
 * sites (engine/modules/compress.cpp:141, core.cpp:1228) compile unchanged
 * when this header replaces "../compress/{thresholdv16,thresholdv,topk}.h".
 * Every call forwards to the C-ABI in stg/codec.h (libstg_codec.so); status
 * codes become std::runtime_error, as the reference throws (topk.cpp:34).
 *
 * compress() keeps the reference's synchronous host-memory contract (src in
 * pinned shm, dst new[]-allocated, compress.cpp:60-64).  compress_device()
 * is the device-resident, asynchronous form for GPU-resident buckets.
 */
#ifndef STG_COMPRESSOR_H
#define STG_COMPRESSOR_H

#include <cstddef>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>

#include "codec.h"

class ThreadPool;  // engine/threadpool.h; the GPU codec never dereferences it

class Compressor {
protected:
    std::unique_ptr<ThreadPool> &thread_pool_;
    std::string name_;
    stg_codec_t h_ = nullptr;

    static int &default_device_ref() {
        static int dev = 0;
        return dev;
    }

public:
    template <typename T = float>
    using Segment = std::pair<T *, size_t>;

    template <typename T = float>
    using ConstSegment = std::pair<const T *, const size_t>;

    /* HIP device the codecs are created on (the node master's GPU). */
    static void set_default_device(int device) { default_device_ref() = device; }

    Compressor(std::unique_ptr<ThreadPool> &thread_pool, std::string name, const char *method)
        : thread_pool_(thread_pool), name_(std::move(name)) {
        if (stg_codec_create(method, default_device_ref(), &h_) != STG_OK) throw std::runtime_error(stg_last_error());
    }
    Compressor(const Compressor &) = delete;
    Compressor &operator=(const Compressor &) = delete;
    virtual ~Compressor() { stg_codec_destroy(h_); }

    inline const std::string &name() { return name_; }

    virtual size_t compress(const std::string &name, ConstSegment<float> src, uint32_t k, Segment<uint32_t> dst_idx,
                            Segment<float> dst_val, int32_t idx_offset = 0) {
        size_t out = 0;
        if (stg_codec_compress_host(h_, name.c_str(), src.first, src.second, k, dst_idx.first, dst_idx.second,
                                    dst_val.first, dst_val.second, idx_offset, &out) != STG_OK)
            throw std::runtime_error(stg_last_error());
        return out;
    }

    /* Device-resident form: all pointers on the codec's device, the pair count
     * lands in *d_count, nothing synchronises. */
    void compress_device(const std::string &name, ConstSegment<float> src, uint32_t k, Segment<uint32_t> dst_idx,
                         Segment<float> dst_val, uint32_t *d_count, void *stream, int32_t idx_offset = 0) {
        if (stg_codec_compress_device(h_, name.c_str(), src.first, src.second, k, dst_idx.first, dst_idx.second,
                                      dst_val.first, dst_val.second, idx_offset, d_count, stream) != STG_OK)
            throw std::runtime_error(stg_last_error());
    }

    /* Batched device-resident form: the engine's per-iteration set of MERGE
     * compress tasks (compress.cpp:141 once per bucket) issued as one call;
     * same results as compress_device on each bucket in order. */
    void compress_batch_device(const stg_bucket_t *buckets, size_t n, void *stream) {
        if (stg_codec_compress_batch_device(h_, buckets, n, stream) != STG_OK)
            throw std::runtime_error(stg_last_error());
    }

    stg_codec_t handle() { return h_; }
};

class ThresholdvCompressor16 : public Compressor {
public:
    bool multicore_;
    ThresholdvCompressor16(std::unique_ptr<ThreadPool> &thread_pool, bool multicore = true)
        : Compressor(thread_pool, "Thresholdv16", "thresholdv16"), multicore_(multicore) {}
};

class ThresholdvCompressor : public Compressor {
public:
    bool multicore_;
    ThresholdvCompressor(std::unique_ptr<ThreadPool> &thread_pool, bool multicore = true)
        : Compressor(thread_pool, "Thresholdv", "thresholdv"), multicore_(multicore) {}
};

class TopkCompressor : public Compressor {
public:
    enum TopkCompressMethod { NTH_ELEMENT_MULTICORE, NTH_ELEMENT, HEAP };
    TopkCompressMethod method_;
    explicit TopkCompressor(std::unique_ptr<ThreadPool> &thread_pool)
        : Compressor(thread_pool, "Topk", "topk"), method_(NTH_ELEMENT) {}
};

#endif /* STG_COMPRESSOR_H */
