/*
 * ref_driver.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Thin extern "C" driver around the *reference's own* codec sources, compiled
 * in place from /root/reference/backend/src by oracle/Makefile into
 * oracle/_ref/libstg_ref.so (git-ignored).  No reference source is copied into
 * this repository.  Used to (1) pin the clean-room restatement
 * (oracle/stg_oracle.cpp) bit-exactly and (2) generate tests/golden/.
 *
 * Reference interface driven: Compressor::compress(name, src, k, dst_idx,
 * dst_val, idx_offset) (compress/compressor.h:30) on ThresholdvCompressor16
 * (thresholdv16.h:9-38), ThresholdvCompressor (thresholdv.h:9-29) and
 * TopkCompressor (topk.h:9-31); SGD::optimize_raw (optim/sgd.cpp:34-263).
 */
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <vector>

// Read-only access to the per-key AIMD state for trajectory goldens.
#define private public
#include "compress/thresholdv16.h"
#include "compress/topk.h"
#undef COMPRESS_RANDOMK_H  // thresholdv.h reuses randomk.h's include guard
#include "compress/thresholdv.h"
#undef private

#define REF_API extern "C" __attribute__((visibility("default")))

namespace {
std::unique_ptr<ThreadPool> g_pool;  // the three codecs never dereference it

struct RefTv {
    ThresholdvCompressor c{g_pool, true};
    // threshold-v keys its state by src pointer: keep one stable buffer per key,
    // as the engine's two alternating shm gradient buffers are (core.cpp:967).
    std::map<unsigned long long, std::vector<float>> buf;
};
}  // namespace

REF_API void *ref_tv16_new(void) { return new ThresholdvCompressor16(g_pool, true); }
REF_API void ref_tv16_free(void *h) { delete static_cast<ThresholdvCompressor16 *>(h); }
REF_API size_t ref_tv16_compress(void *h, const char *name, const float *src, size_t n, uint32_t k,
                                 uint32_t *idx, size_t idx_cap, float *val, int32_t idx_offset) {
    auto *c = static_cast<ThresholdvCompressor16 *>(h);
    return c->compress(name, std::make_pair(src, n), k, std::make_pair(idx, idx_cap),
                       std::make_pair(val, idx_cap), idx_offset);
}
REF_API int ref_tv16_state(void *h, const char *name, float *t, float *inc) {
    auto *c = static_cast<ThresholdvCompressor16 *>(h);
    auto it = c->threshold_map_.find(name);
    if (it == c->threshold_map_.end()) return -1;
    *t = it->second;
    *inc = c->threshold_map_inc_[name];
    return 0;
}

REF_API void *ref_tv_new(void) { return new RefTv(); }
REF_API void ref_tv_free(void *h) { delete static_cast<RefTv *>(h); }
REF_API size_t ref_tv_compress(void *h, unsigned long long key, const float *src, size_t n, uint32_t k,
                               uint32_t *idx, size_t cap, float *val) {
    auto *r = static_cast<RefTv *>(h);
    auto &b = r->buf[key];
    if (b.size() != n) b.assign(n, 0.f);
    std::memcpy(b.data(), src, n * sizeof(float));
    return r->c.compress("", std::make_pair(static_cast<const float *>(b.data()), n), k,
                         std::make_pair(idx, cap), std::make_pair(val, cap), 0);
}
REF_API int ref_tv_state(void *h, unsigned long long key, float *t) {
    auto *r = static_cast<RefTv *>(h);
    auto bit = r->buf.find(key);
    if (bit == r->buf.end()) return -1;
    auto it = r->c.threshold_map_.find(reinterpret_cast<uintptr_t>(bit->second.data()));
    if (it == r->c.threshold_map_.end()) return -1;
    *t = it->second;
    return 0;
}

REF_API long long ref_topk_compress(const float *src, size_t n, uint32_t k, uint32_t *idx, size_t cap,
                                    float *val) {
    TopkCompressor c(g_pool);
    try {
        return static_cast<long long>(
            c.compress("", std::make_pair(src, n), k, std::make_pair(idx, cap), std::make_pair(val, cap), 0));
    } catch (const std::exception &) {
        return -1;
    }
}
