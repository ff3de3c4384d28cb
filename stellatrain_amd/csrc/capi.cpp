// capi.cpp -- host side of the C-ABI declared in include/stg/codec.h.
//
// Owns: codec handles (method, device), the per-key AIMD state slots (device
// resident, 16 B each, in never-moving chunks), and one workspace per HIP
// stream.  The reference keeps the threshold maps in the compressor object
// behind a mutex (thresholdv16.h:11-14, thresholdv16.cpp:84-91,255-258) and
// is called concurrently from up to 32 ThreadPool workers on different keys
// (engine/config.h:7, core_module_api.cpp:7-24); here every call locks the
// handle only to look up its slot and its stream's workspace, and the launch
// sequence of one call holds that workspace's lock so calls sharing a stream
// cannot interleave their kernels.
#include <cmath>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include <dlfcn.h>

#include "../../include/stg/codec.h"
#include "ws.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

#define HIP_TRY(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(STG_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

enum Method { M_TV16 = 0, M_TV = 1, M_TOPK = 2, M_TOPK_EXACT = 3 };

constexpr uint32_t SLOTS_PER_CHUNK = 4096;

struct Workspace {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    stg::DevWS d{};
    void *fixed = nullptr;
    size_t cap_sums = 0, cap_tiles = 0, cap_stage = 0, cap_desc = 0, cap_lone = 0;
    uint32_t epoch = 0;  // thresholdv16 call counter (hand-off tags)
    uint32_t tk_tag = 0; // one-launch top-k call counter (topk1.hip)
    uint32_t lone_calls = 0;  // thresholdv16 one-bucket path calls (tv16.hip: parity of its per-call blocks)
    // threshold-v: the ticket's value at the next call, the last call's
    // range-descriptor tag and the descriptor block last zeroed (tile_cnt, its size)
    uint64_t tv_base = 0;
    uint32_t tv_tag = 0;
    uint32_t *tv_desc = nullptr;
    size_t tv_desc_cap = 0;
    // device buffers of the host-memory entry point
    float *h_src = nullptr;
    size_t cap_src = 0;
    uint32_t *h_idx = nullptr;
    float *h_val = nullptr;
    size_t cap_out = 0;
    uint32_t *h_count = nullptr;
    uint32_t *pinned_count = nullptr;
    // one-bucket wire path staging (stg_codec_compress_wire_batch_device)
    std::mutex wire_mu;
    uint32_t *wst_pos = nullptr;
    float *wst_val = nullptr;
    size_t cap_wst = 0;

    ~Workspace() {
        (void)hipSetDevice(device);
        if (stream) (void)hipStreamSynchronize(stream);
        (void)hipFree(fixed);
        (void)hipFree(d.sums);
        (void)hipFree(d.desc);
        (void)hipFree(d.tile_cnt);
        (void)hipFree(d.tile_aux);
        (void)hipFree(d.stage_pos);
        (void)hipFree(d.stage_val);
        (void)hipFree(d.ldesc);
        (void)hipFree(d.lq);
        (void)hipFree(d.lw);
        (void)hipFree(d.lv);
        (void)hipFree(h_src);
        (void)hipFree(h_idx);
        (void)hipFree(h_val);
        (void)hipFree(h_count);
        (void)hipFree(wst_pos);
        (void)hipFree(wst_val);
        if (pinned_count) (void)hipHostFree(pinned_count);
    }

    int init() {
        size_t off = 0;
        auto carve = [&](size_t bytes) {
            const size_t o = off;
            off = (off + bytes + 255) & ~size_t(255);
            return o;
        };
        const size_t o_ctl = carve(sizeof(stg::FillCtl));
        const size_t o_cp = carve(sizeof(stg::CallParams));
        const size_t o_rs = carve(sizeof(stg::RSel));
        const size_t o_fail = carve(sizeof(uint32_t));
        const size_t o_cand = carve(sizeof(uint32_t) * stg::CAND_WORDS * stg::MAX_BATCH);
        const size_t o_misc = carve(sizeof(uint32_t) * 64);
        const size_t o_tvt = carve(sizeof(uint64_t));
        const size_t o_wh = carve(sizeof(uint32_t) * 2 * stg::LNBIN);
        const size_t o_larr = carve(sizeof(uint32_t) * stg::LARR_WORDS);
        const size_t o_we = carve(sizeof(uint2) * stg::LNBIN * stg::LBCAP);
        const size_t o_crew = carve(sizeof(stg::CrewCtl) * stg::MAX_BATCH);
        const size_t o_tkc = carve(sizeof(stg::TopkCtl) * 2);
        const size_t o_tkf = carve(sizeof(uint32_t) * 2 * stg::TK2_FINE);
        HIP_TRY(hipMalloc(&fixed, off));
        // zeroed on this workspace's stream: the launches that read the
        // control block are ordered after it (a plain hipMemset runs on the
        // null stream, which a non-blocking stream does not wait for)
        HIP_TRY(hipMemsetAsync(fixed, 0, off, stream));
        char *b = static_cast<char *>(fixed);
        d.ctl = reinterpret_cast<stg::FillCtl *>(b + o_ctl);
        d.cp = reinterpret_cast<stg::CallParams *>(b + o_cp);
        d.rsel = reinterpret_cast<stg::RSel *>(b + o_rs);
        d.fail = reinterpret_cast<uint32_t *>(b + o_fail);
        d.cand = reinterpret_cast<uint32_t *>(b + o_cand);
        d.misc = reinterpret_cast<uint32_t *>(b + o_misc);
        d.tv_ticket = reinterpret_cast<uint64_t *>(b + o_tvt);
        d.whist = reinterpret_cast<uint32_t *>(b + o_wh);
        d.larr = reinterpret_cast<uint32_t *>(b + o_larr);
        d.went = reinterpret_cast<uint2 *>(b + o_we);
        d.crew = reinterpret_cast<stg::CrewCtl *>(b + o_crew);
        d.tkctl = reinterpret_cast<stg::TopkCtl *>(b + o_tkc);
        d.tkfine = reinterpret_cast<uint32_t *>(b + o_tkf);
        return STG_OK;
    }

    // Grow-only scratch.  Growing waits for this stream's in-flight work.
    template <typename T>
    int grow(T *&p, size_t &cap, size_t need) {
        if (need <= cap) return STG_OK;
        HIP_TRY(hipStreamSynchronize(stream));
        (void)hipFree(p);
        p = nullptr;
        const size_t n = std::max<size_t>(need, cap + cap / 2);
        HIP_TRY(hipMalloc(&p, n * sizeof(T)));
        cap = n;
        return STG_OK;
    }

    // thresholdv16 chunk descriptors: zeroed on (re)allocation, so no stale
    // word carries a live call tag (epochs start at 1)
    int ensure_desc(size_t n) {
        if (n <= cap_desc) return STG_OK;
        int rc;
        if ((rc = grow(d.desc, cap_desc, n))) return rc;
        HIP_TRY(hipMemsetAsync(d.desc, 0, cap_desc * sizeof(stg::ChunkDesc), stream));
        return STG_OK;
    }

    // one-bucket path lists (tv16lone.hip): per chunk a tagged count pair and
    // the qualifying / window line lists.  The finish inside the scan launch
    // (tv16lf2.h) POLLS the count pairs while chunks are still being listed and
    // takes a pair as this call's once its high word equals the call tag, so
    // the pairs are zeroed on (re)allocation: recycled device memory (a freed
    // workspace's pairs, whose tags restart at 1 in every workspace) could
    // otherwise already hold a live tag with another call's counts.  Tags are
    // >= 1 and only this workspace writes its pairs afterwards, so no stale
    // pair ever matches a later call.  The lists themselves are read only
    // behind a matched pair.
    int ensure_lone(size_t nc) {
        if (nc <= cap_lone) return STG_OK;
        HIP_TRY(hipStreamSynchronize(stream));
        (void)hipFree(d.ldesc);
        (void)hipFree(d.lq);
        (void)hipFree(d.lw);
        (void)hipFree(d.lv);
        d.ldesc = nullptr;
        d.lq = nullptr;
        d.lw = nullptr;
        d.lv = nullptr;
        const size_t c = std::min<size_t>(stg::LMAXC, std::max(nc, cap_lone + cap_lone / 2));
        cap_lone = 0;
        HIP_TRY(hipMalloc(&d.ldesc, c * sizeof(uint2)));
        HIP_TRY(hipMalloc(&d.lq, c * stg::LQCAP * sizeof(uint32_t)));
        HIP_TRY(hipMalloc(&d.lw, c * stg::LWCAP * sizeof(uint2)));
        HIP_TRY(hipMalloc(&d.lv, c * stg::LQCAP * 4 * sizeof(float4)));
        static const bool stale = getenv("STG_DEBUG_LDESC_STALE") && atoi(getenv("STG_DEBUG_LDESC_STALE")) == 1;
        if (stale) {  // diagnostics: what a recycled block looks like (every pair tagged 1..8, counts 0)
            std::vector<uint2> p(c);
            for (size_t i = 0; i < c; ++i) p[i] = make_uint2(0u, 1u + (uint32_t)(i & 7u));
            HIP_TRY(hipMemcpyAsync(d.ldesc, p.data(), c * sizeof(uint2), hipMemcpyHostToDevice, stream));
            HIP_TRY(hipStreamSynchronize(stream));
        } else {
            HIP_TRY(hipMemsetAsync(d.ldesc, 0, c * sizeof(uint2), stream));
        }
        cap_lone = c;
        return STG_OK;
    }

    int ensure_wire_stage(size_t n) {  // (caller holds wire_mu)
        size_t c = cap_wst;
        int rc;
        if ((rc = grow(wst_pos, c, n))) return rc;
        c = cap_wst;
        if ((rc = grow(wst_val, c, n))) return rc;
        cap_wst = c;
        return STG_OK;
    }

    int ensure(size_t sums, size_t tiles, size_t stage) {
        int rc;
        if ((rc = grow(d.sums, cap_sums, sums))) return rc;
        size_t ct = cap_tiles;
        if ((rc = grow(d.tile_cnt, ct, tiles))) return rc;
        ct = cap_tiles;
        if ((rc = grow(d.tile_aux, ct, tiles))) return rc;
        cap_tiles = ct;
        size_t cs = cap_stage;
        if ((rc = grow(d.stage_pos, cs, stage))) return rc;
        cs = cap_stage;
        if ((rc = grow(d.stage_val, cs, stage))) return rc;
        cap_stage = cs;
        return STG_OK;
    }
};

}  // namespace

struct stg_codec {
    Method method;
    int device = 0;
    int num_cu = 256;
    std::string name;
    std::mutex mu;
    std::unordered_map<std::string, uint32_t> slot_of;
    std::vector<KeyState *> chunks;
    uint32_t nslots = 0;
    std::unordered_map<hipStream_t, std::unique_ptr<Workspace>> ws;
    // kernel timing (stg_codec_set_timing)
    bool timing = false;
    std::vector<std::array<hipEvent_t, 3>> ev_pending, ev_pool;
    double ms_acc[3] = {0, 0, 0};
    uint64_t timed_calls = 0;

    ~stg_codec() {
        (void)hipSetDevice(device);
        ws.clear();
        for (auto *c : chunks) (void)hipFree(c);
        for (auto *v : {&ev_pending, &ev_pool})
            for (auto &e : *v)
                for (auto x : e) (void)hipEventDestroy(x);
    }

    // Events for one timed call (nullptr when timing is off).
    int take_events(std::array<hipEvent_t, 3> *e, bool *on) {
        std::lock_guard<std::mutex> g(mu);
        *on = timing;
        if (!timing) return STG_OK;
        if (!ev_pool.empty()) { *e = ev_pool.back(); ev_pool.pop_back(); }
        else for (auto &x : *e) HIP_TRY(hipEventCreate(&x));
        ev_pending.push_back(*e);
        return STG_OK;
    }

    KeyState *slot_ptr(uint32_t s) { return chunks[s / SLOTS_PER_CHUNK] + (s % SLOTS_PER_CHUNK); }

    // Returns the state slot of `key`; *fresh = true when it was just created.
    int slot(const std::string &key, KeyState **out, bool *fresh) {
        std::lock_guard<std::mutex> g(mu);
        auto it = slot_of.find(key);
        if (it != slot_of.end()) { *out = slot_ptr(it->second); *fresh = false; return STG_OK; }
        if (nslots % SLOTS_PER_CHUNK == 0) {
            KeyState *c = nullptr;
            HIP_TRY(hipMalloc(&c, sizeof(KeyState) * SLOTS_PER_CHUNK));
            // states are read on any stream: zero them before any launch sees them
            HIP_TRY(hipMemsetAsync(c, 0, sizeof(KeyState) * SLOTS_PER_CHUNK, nullptr));
            HIP_TRY(hipStreamSynchronize(nullptr));
            chunks.push_back(c);
        }
        const uint32_t s = nslots++;
        slot_of.emplace(key, s);
        *out = slot_ptr(s);
        *fresh = true;
        return STG_OK;
    }

    int workspace(hipStream_t s, Workspace **out) {
        std::lock_guard<std::mutex> g(mu);
        auto it = ws.find(s);
        if (it != ws.end()) { *out = it->second.get(); return STG_OK; }
        auto w = std::make_unique<Workspace>();
        w->device = device;
        w->stream = s;
        int rc = w->init();
        if (rc) return rc;
        *out = w.get();
        ws.emplace(s, std::move(w));
        return STG_OK;
    }
};

struct stg_sgd {
    int device = 0;
    float lr, momentum, dampening, weight_decay;
    bool nesterov, maximize;
    uint32_t iter = 0;
    std::mutex mu;
    std::unordered_map<std::string, std::pair<float *, uint32_t>> mom;
    ~stg_sgd() {
        (void)hipSetDevice(device);
        for (auto &kv : mom) (void)hipFree(kv.second.first);
    }
};

struct stg_adam {
    int device = 0;
    uint32_t *fail = nullptr;  // device failure word (amsgrad look-back timeout)
    float lr, b1, b2, eps, weight_decay;
    bool amsgrad, maximize;
    struct Name {
        float *m = nullptr, *v = nullptr, *vmax = nullptr;
        uint32_t *tiles = nullptr;  // amsgrad look-back words, one uint64 per ADAM_TILE of param_len
        uint32_t len = 0, tick = 1;
    };
    std::mutex mu;
    std::unordered_map<std::string, Name> st;
    ~stg_adam() {
        (void)hipSetDevice(device);
        (void)hipFree(fail);
        for (auto &kv : st) {
            (void)hipFree(kv.second.m);
            (void)hipFree(kv.second.tiles);
        }
    }
};

namespace {

std::string state_key(Method m, const char *key, const void *src) {
    if (m == M_TV) {  // thresholdv.cpp:44: keyed by the src pointer
        char b[32];
        snprintf(b, sizeof b, "\x01%p", src);
        return b;
    }
    return key ? std::string(key) : std::string();
}

// Device-wide admission of thresholdv16 launches.  No launch waits on a
// workgroup that is not running (chunks are taken dynamically), so admission
// is a throughput policy, not a correctness one.  (Scans one at a time per
// device, each waiting for the previous one's on another stream, measured
// slower: profiles/r02_streams.jsonl.)
//  * STG_TV16_INFLIGHT (1-4; default unlimited) launches per device in
//    flight: a launch on stream s first makes s wait for the oldest in-flight
//    launch of another stream when the lane is full.  Unlimited (the default)
//    records no events at all: concurrent callers on their own streams
//    overlap freely (the reference's per-task compress() from many pool
//    workers, engine/modules/compress.cpp:141, core_module_api.cpp:7-24).
struct FusedLane {
    std::mutex mu;
    std::vector<std::pair<hipEvent_t, hipStream_t>> inflight;  // oldest first
    std::vector<hipEvent_t> pool;
};

FusedLane g_lanes[64];

uint32_t fused_inflight() {  // 0: unlimited
    static const uint32_t v = [] {
        if (const char *e = getenv("STG_TV16_INFLIGHT")) {
            const int x = atoi(e);
            return x <= 0 ? 0u : (uint32_t)std::min(4, x);
        }
        return 0u;
    }();
    return v;
}

thread_local std::unordered_map<int, hipStream_t> t_streams;

int thread_stream(int device, hipStream_t *s) {
    auto it = t_streams.find(device);
    if (it != t_streams.end()) { *s = it->second; return STG_OK; }
    hipStream_t st;
    HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    t_streams.emplace(device, st);
    *s = st;
    return STG_OK;
}

int validate(const stg_codec *h, size_t n, uint32_t k, size_t idx_cap, size_t val_cap, const uint32_t *d_count) {
    if (val_cap < idx_cap) return fail(STG_ERR_INVALID, "value capacity smaller than index capacity");
    if ((h->method == M_TOPK || h->method == M_TOPK_EXACT) && idx_cap < k)
        return fail(STG_ERR_INVALID, "Invalid parameter k");  // topk.cpp:33-34
    if (n >= (size_t(1) << 32) || idx_cap >= (size_t(1) << 32))
        return fail(STG_ERR_UNSUPPORTED, "bucket larger than 2^32-1 elements (uint32 indices)");
    if (!d_count) return fail(STG_ERR_INVALID, "null count pointer");
    return STG_OK;
}

// One thresholdv16 launch over `nb` buckets with distinct keys (caller holds
// ws->mu).  Scratch is carved per bucket from ws->d.sums: the first-threshold
// line sums, later the fill's candidate heap (two words per line).
int launch_tv16_group(stg_codec *h, Workspace *ws, std::vector<stg::Tv16Bucket> &grp, hipStream_t s) {
    if (grp.empty()) return STG_OK;
    size_t need = 0;
    for (auto &b : grp) need += 2 * ((b.n + 15) / 16 + 64);
    int rc;
    if ((rc = ws->ensure(need, 1, 1))) return rc;
    size_t off = 0, chunks = 0;
    for (auto &b : grp) {
        b.sums = ws->d.sums + off;
        off += 2 * ((b.n + 15) / 16 + 64);
        chunks += std::max<size_t>(1, (b.n / 16 + stg::TV16_CHUNK - 1) / stg::TV16_CHUNK);
    }
    if ((rc = ws->ensure_desc(chunks))) return rc;
    if (grp.size() == 1) {  // the one-bucket path's lists (tv16lone.hip), in its own chunks
        const size_t lc = std::max<size_t>(1, (grp[0].n / 16 + stg::LCHUNK - 1) / stg::LCHUNK);
        if (lc <= stg::LMAXC && (rc = ws->ensure_lone(lc))) return rc;
    }
    std::array<hipEvent_t, 3> evs{};
    bool timed = false;
    if ((rc = h->take_events(&evs, &timed))) return rc;
    // 24-bit call epochs tag every hand-off word ({epoch:24 | kind:8});
    // epoch parity selects the per-call counters.  On wrap, clear the blocks.
    if (++ws->epoch >= (1u << 24)) {
        ws->epoch = 1;
        HIP_TRY(hipMemsetAsync(ws->d.ctl, 0, sizeof(stg::FillCtl), s));
        HIP_TRY(hipMemsetAsync(ws->d.desc, 0, ws->cap_desc * sizeof(stg::ChunkDesc), s));
    }
    stg::Tv16Launch a{};
    a.b = grp.data();
    a.nb = (uint32_t)grp.size();
    a.num_cu = h->num_cu;
    a.ev = timed ? evs.data() : nullptr;
    a.epoch = ws->epoch;
    // Workgroups are dealt round-robin over the 8 XCDs (32 CUs, 64 slots
    // each): a launch's share is a multiple of 8 so every XCD holds the same
    // number of each launch's workgroups.
    const uint32_t inflight = fused_inflight();
    constexpr uint32_t XCDS = 8;
    // Every launch may use the whole chip (two scan workgroups per CU): with
    // dynamic chunk takes, the workgroups of concurrent launches simply
    // interleave as slots free up (an even split of the slots between the
    // in-flight launches measured no faster).
    a.max_wg = (uint32_t)(2 * h->num_cu);
    (void)XCDS;
    a.desc_cap = (uint32_t)std::min<size_t>(ws->cap_desc, 0xffffffffu);
    a.lone_cap = (uint32_t)ws->cap_lone;
    a.lone_calls = &ws->lone_calls;
    if (!inflight) {  // no admission: nothing to track
        HIP_TRY(stg::launch_tv16(a, ws->d, s));
        grp.clear();
        return STG_OK;
    }
    FusedLane &lane = g_lanes[h->device & 63];
    std::lock_guard<std::mutex> lg(lane.mu);
    const size_t max_inflight = inflight;
    while (lane.inflight.size() >= max_inflight) {
        auto old = lane.inflight.front();
        lane.inflight.erase(lane.inflight.begin());
        if (old.second != s) HIP_TRY(hipStreamWaitEvent(s, old.first, 0));
        lane.pool.push_back(old.first);
    }
    HIP_TRY(stg::launch_tv16(a, ws->d, s));
    hipEvent_t done;
    if (!lane.pool.empty()) { done = lane.pool.back(); lane.pool.pop_back(); }
    else HIP_TRY(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(done, s));
    lane.inflight.emplace_back(done, s);
    grp.clear();
    return STG_OK;
}

// thresholdv16 over a sequence of buckets: runs of distinct keys (<= 16)
// share one launch; the per-key state makes a repeated key wait for the
// launch that updates it.
int run_tv16(stg_codec *h, const stg_bucket_t *bk, size_t nbk, hipStream_t s, float *const *resid = nullptr,
             const stg::GatherArgs *gather = nullptr, const int *wire_flags = nullptr) {
    HIP_TRY(hipSetDevice(h->device));
    Workspace *ws = nullptr;
    int rc = h->workspace(s, &ws);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(ws->mu);
    std::vector<stg::Tv16Bucket> grp;
    grp.reserve(stg::MAX_BATCH);
    for (size_t i = 0; i < nbk; ++i) {
        const stg_bucket_t &b = bk[i];
        if (b.n == 0) {
            HIP_TRY(hipMemsetAsync(b.d_count, 0, sizeof(uint32_t), s));
            continue;
        }
        KeyState *st;
        bool fresh;
        if ((rc = h->slot(state_key(h->method, b.key, b.d_src), &st, &fresh))) return rc;
        bool dup = false;
        for (auto &x : grp) dup |= x.state == st;
        if (dup || grp.size() == stg::MAX_BATCH)
            if ((rc = launch_tv16_group(h, ws, grp, s))) return rc;
        stg::Tv16Bucket t{};
        t.src = b.d_src;
        t.n = b.n;
        t.k = b.k;
        t.dst_len = (uint32_t)b.idx_cap;
        t.idx = b.d_idx;
        t.val = b.d_val;
        t.idx_offset = b.idx_offset;
        t.count_out = b.d_count;
        t.state = st;
        t.first = fresh;
        t.resid = resid ? resid[i] : nullptr;
        t.gather = i == 0 ? gather : nullptr;
        t.wflag = wire_flags ? (uint32_t)wire_flags[i] & 3u : 0u;
        grp.push_back(t);
    }
    return launch_tv16_group(h, ws, grp, s);
}

// ModuleCompress::run MERGE error feedback (compress.cpp:172-186) after the
// codec: the ragged tail (not streamed by the fused kernel) is copied, then the
// numel = idx_cap selected slots are zeroed in the bucket and the residual.
int ef_after(stg_codec *h, const stg_bucket_t &b, float *resid, bool fused, hipStream_t s) {
    float *g = const_cast<float *>(b.d_src);
    if (!fused) {
        HIP_TRY(stg::launch_error_feedback(g, b.n, b.d_idx, b.idx_cap, resid, h->num_cu, s));
        return STG_OK;
    }
    const size_t full = b.n / 16 * 16;
    if (b.n > full)
        HIP_TRY(hipMemcpyAsync(resid + full, g + full, (b.n - full) * sizeof(float), hipMemcpyDeviceToDevice, s));
    HIP_TRY(stg::launch_ef_zero(g, resid, b.d_idx, b.idx_cap, b.n, h->num_cu, s));
    return STG_OK;
}


int run_device(stg_codec *h, const char *key, const float *d_src, const void *key_ptr, size_t n, uint32_t k,
               uint32_t *d_idx, size_t idx_cap, float *d_val, size_t val_cap, int32_t idx_offset, uint32_t *d_count,
               hipStream_t s) {
    if (!h) return fail(STG_ERR_INVALID, "null codec handle");
    int rc = validate(h, n, k, idx_cap, val_cap, d_count);
    if (rc) return rc;
    if (h->method == M_TV16) {
        const stg_bucket_t b{key, d_src, n, k, d_idx, idx_cap, d_val, val_cap, idx_offset, d_count};
        return run_tv16(h, &b, 1, s);
    }
    HIP_TRY(hipSetDevice(h->device));
    Workspace *ws = nullptr;
    if ((rc = h->workspace(s, &ws))) return rc;
    std::lock_guard<std::mutex> g(ws->mu);
    if (n == 0) {
        HIP_TRY(hipMemsetAsync(d_count, 0, sizeof(uint32_t), s));
        return STG_OK;
    }
    std::array<hipEvent_t, 3> evs{};
    bool timed = false;
    if ((rc = h->take_events(&evs, &timed))) return rc;
    hipEvent_t *ev = timed ? evs.data() : nullptr;
    if (h->method == M_TV) {
        KeyState *st;
        bool fresh;
        if ((rc = h->slot(state_key(h->method, key, key_ptr), &st, &fresh))) return rc;
        // range descriptors (tv.hip): counts at tile_cnt, maxima at tile_aux, two words per range
        if ((rc = ws->ensure(1, 2 * (size_t)stg::TV_MAXG, 1))) return rc;
        if (ws->tv_desc != ws->d.tile_cnt || ws->tv_desc_cap != ws->cap_tiles) {  // fresh memory: no stale tags
            HIP_TRY(hipMemsetAsync(ws->d.tile_cnt, 0, ws->cap_tiles * sizeof(uint32_t), s));
            HIP_TRY(hipMemsetAsync(ws->d.tile_aux, 0, ws->cap_tiles * sizeof(uint32_t), s));
            ws->tv_desc = ws->d.tile_cnt;
            ws->tv_desc_cap = ws->cap_tiles;
        }
        if (++ws->tv_tag == 0) ws->tv_tag = 1;
        uint32_t grid = 0;
        stg::TvLaunch a{d_src, n, k, (uint32_t)idx_cap, d_idx, d_val, d_count, st, fresh, h->num_cu, ev,
                        ws->tv_tag, ws->tv_base, &grid};
        HIP_TRY(stg::launch_tv(a, ws->d, s));
        ws->tv_base += grid;
    } else {
        const size_t ntiles = (n + stg::TV_TILE - 1) / stg::TV_TILE;
        // superset entries (two words each, stg::TOPK_SUP_CAP per tile); per-tile
        // counts, their prefixes and the superset counts
        // + the level-2 bin's list (two words per key)
        // (whole groups of TK2_REG tiles: topk1.hip's fixed superset slots)
        const size_t stiles = (ntiles + stg::TK2_REG - 1) / stg::TK2_REG * stg::TK2_REG;
        if ((rc = ws->ensure(2 * stiles * stg::TOPK_SUP_CAP + 2 * stg::TOPK_LIST_CAP, 3 * ntiles + 1, 1))) return rc;
        stg::TopkLaunch a{d_src, n, k, (uint32_t)idx_cap, d_idx, d_val, idx_offset, h->method == M_TOPK, d_count,
                          h->num_cu, ev};
        const size_t m = h->method == M_TOPK ? (n + 3) / 4 : n;
        if ((m + stg::TV_TILE - 1) / stg::TV_TILE <= stg::TOPK_LIST_TILES) {
            // one launch, steered by the key's last k-th magnitude (its first call: the select inside it)
            KeyState *st;
            bool fresh;
            if ((rc = h->slot(state_key(h->method, key, key_ptr), &st, &fresh))) return rc;
            HIP_TRY(stg::launch_topk1(a, ws->d, st, !fresh, &ws->tk_tag, s));
        } else {
            HIP_TRY(stg::launch_topk(a, ws->d, s));
        }
    }
    return STG_OK;
}

// MERGE decompress scratch, one per (device, stream): the per-tile counts and
// the u32 winner words (zero between calls).  Keyed like the codec
// workspaces, so merges issued from one thread on several streams or devices
// never share scratch.  Growing waits for the stream's in-flight work.
struct MergeScratch {
    std::mutex mu;
    int device = 0;
    uint32_t *tiles = nullptr, *win = nullptr;
    size_t cap_tiles = 0, cap_win = 0;
    // world == 1 in one launch: tagged per-tile counts (cap_tiles of them, zeroed
    // whenever reallocated); the tile ticket and the duplicate flag
    uint64_t *desc = nullptr, *ticket = nullptr;
    uint32_t tag = 0;
    uint32_t *fail = nullptr;  // sticky device failure word (a look-back that gave up)
    ~MergeScratch() {
        (void)hipSetDevice(device);
        (void)hipFree(tiles);
        (void)hipFree(win);
        (void)hipFree(desc);
        (void)hipFree(ticket);
        (void)hipFree(fail);
    }
};
std::mutex g_merge_mu;
// shared: a caller holds its reference for the whole call, so a concurrent
// stg_scatter_merge_release never frees a scratch another thread has looked up
std::map<std::pair<int, hipStream_t>, std::shared_ptr<MergeScratch>> g_merge;

std::shared_ptr<MergeScratch> merge_scratch(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> g(g_merge_mu);
    auto &slot = g_merge[{dev, s}];
    if (!slot) { slot = std::make_shared<MergeScratch>(); slot->device = dev; }
    return slot;
}

// Caller holds m->mu.
int merge_scratch_ensure(MergeScratch *m, hipStream_t s, size_t n, size_t per_rank, int world) {
    // per-tile counts and their prefixes (the world > 1 mark scan)
    // ... and the world-1 emission's tagged tile counts (tiles of >= MERGE_TILE / 16 pairs)
    const size_t tiles = std::max(2 * ((std::max(n, per_rank) + stg::MERGE_TILE - 1) / stg::MERGE_TILE) + 2,
                                  (per_rank + stg::MERGE_TILE / 16 - 1) / (stg::MERGE_TILE / 16) + 2);
    if (tiles > m->cap_tiles) {
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(m->tiles);
        m->tiles = nullptr;
        HIP_TRY(hipMalloc(&m->tiles, tiles * sizeof(uint32_t)));
        (void)hipFree(m->desc);
        m->desc = nullptr;
        HIP_TRY(hipMalloc(&m->desc, tiles * sizeof(uint64_t)));
        HIP_TRY(hipMemsetAsync(m->desc, 0, tiles * sizeof(uint64_t), s));  // no stale tags
        m->cap_tiles = tiles;
    }
    if (!m->ticket) {  // [0]: the emission's tile ticket; [1]: the duplicate flag (low word)
        HIP_TRY(hipMalloc(&m->ticket, 2 * sizeof(uint64_t)));
        HIP_TRY(hipMemsetAsync(m->ticket, 0, 2 * sizeof(uint64_t), s));
    }
    if (!m->fail) {  // [0] sticky failure bits, [1] the tag of the last call that failed
        HIP_TRY(hipMalloc(&m->fail, 2 * sizeof(uint32_t)));
        HIP_TRY(hipMemsetAsync(m->fail, 0, 2 * sizeof(uint32_t), s));
    }
    const size_t words = std::max<size_t>(world > 1 ? 2 * n : n, 1);  // world > 1: two election halves
    if (words > m->cap_win) {
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(m->win);
        m->win = nullptr;
        const size_t c = std::max(words, m->cap_win + m->cap_win / 2);
        HIP_TRY(hipMalloc(&m->win, c * sizeof(uint32_t)));
        HIP_TRY(hipMemsetAsync(m->win, 0, c * sizeof(uint32_t), s));
        m->cap_win = c;
    }
    return STG_OK;
}

}  // namespace

extern "C" {

const char *stg_last_error(void) { return g_err.c_str(); }

int stg_codec_create(const char *method, int device, stg_codec_t *out) {
    if (!method || !out) return fail(STG_ERR_INVALID, "null argument");
    const std::string m(method);
    auto h = std::make_unique<stg_codec>();
    if (m == "thresholdv16") { h->method = M_TV16; h->name = "Thresholdv16"; }
    else if (m == "thresholdv") { h->method = M_TV; h->name = "Thresholdv"; }
    else if (m == "topk") { h->method = M_TOPK; h->name = "Topk"; }
    else if (m == "topk_exact") { h->method = M_TOPK_EXACT; h->name = "Topk"; }
    else return fail(STG_ERR_UNKNOWN, "Unknown compression method " + m + ".");  // core.cpp:117
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(STG_ERR_INVALID, "no such HIP device");
    h->device = device;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipDeviceGetAttribute(&h->num_cu, hipDeviceAttributeMultiprocessorCount, device));
    *out = h.release();
    return STG_OK;
}

int stg_codec_destroy(stg_codec_t h) {
    delete h;
    return STG_OK;
}

const char *stg_codec_name(stg_codec_t h) { return h ? h->name.c_str() : ""; }

namespace {
// The reference times each compress task as "CRIT_PATH_compress"
// (engine/modules/compress.cpp:140-142, record_stat_start/end).  With
// STG_ROCTX=1 every compress entry point is a roctx range of that name, so
// `rocprofv3 --marker-trace --kernel-trace` shows the host side of each call
// next to its kernels.
struct CritPath {
    // the roctx library is opened only when STG_ROCTX=1 (no link-time
    // dependency on rocprofiler-sdk for an opt-in diagnostic); a missing
    // library leaves the ranges off
    typedef int (*push_fn)(const char *);
    typedef int (*pop_fn)();
    struct Api {
        push_fn push = nullptr;
        pop_fn pop = nullptr;
    };
    const Api &api;
    CritPath() : api(get()) {
        if (api.push) api.push("CRIT_PATH_compress");
    }
    ~CritPath() {
        if (api.pop) api.pop();
    }
    static const Api &get() {
        static const Api a = [] {
            Api r;
            if (!(getenv("STG_ROCTX") && atoi(getenv("STG_ROCTX")) == 1)) return r;
            void *h = dlopen("librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_GLOBAL);
            if (!h) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so", RTLD_NOW | RTLD_GLOBAL);
            if (!h) return r;
            r.push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
            r.pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
            if (!r.push || !r.pop) r = Api{};
            return r;
        }();
        return a;
    }
};
}  // namespace

int stg_codec_compress_device(stg_codec_t h, const char *key, const float *d_src, size_t n, uint32_t k,
                              uint32_t *d_idx, size_t idx_cap, float *d_val, size_t val_cap, int32_t idx_offset,
                              uint32_t *d_count, void *stream) {
    CritPath crit_path;
    return run_device(h, key, d_src, d_src, n, k, d_idx, idx_cap, d_val, val_cap, idx_offset, d_count,
                      static_cast<hipStream_t>(stream));
}

int stg_codec_compress_batch_device(stg_codec_t h, const stg_bucket_t *buckets, size_t nbuckets, void *stream) {
    CritPath crit_path;
    if (!h) return fail(STG_ERR_INVALID, "null codec handle");
    if (nbuckets && !buckets) return fail(STG_ERR_INVALID, "null bucket array");
    for (size_t i = 0; i < nbuckets; ++i) {
        const stg_bucket_t &b = buckets[i];
        const int rc = validate(h, b.n, b.k, b.idx_cap, b.val_cap, b.d_count);
        if (rc) return rc;
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (h->method == M_TV16) return run_tv16(h, buckets, nbuckets, s);
    for (size_t i = 0; i < nbuckets; ++i) {
        const stg_bucket_t &b = buckets[i];
        const int rc = run_device(h, b.key, b.d_src, b.d_src, b.n, b.k, b.d_idx, b.idx_cap, b.d_val, b.val_cap,
                                  b.idx_offset, b.d_count, s);
        if (rc) return rc;
    }
    return STG_OK;
}

int stg_merge_compress_batch_device(stg_codec_t h, const stg_bucket_t *buckets, float *const *d_residuals,
                                    size_t nbuckets, void *stream) {
    CritPath crit_path;
    if (!h) return fail(STG_ERR_INVALID, "null codec handle");
    if (nbuckets && (!buckets || !d_residuals)) return fail(STG_ERR_INVALID, "null bucket or residual array");
    for (size_t i = 0; i < nbuckets; ++i) {
        const stg_bucket_t &b = buckets[i];
        const int rc = validate(h, b.n, b.k, b.idx_cap, b.val_cap, b.d_count);
        if (rc) return rc;
        if (b.n && !d_residuals[i]) return fail(STG_ERR_INVALID, "null residual");
    }
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    const bool fused = h->method == M_TV16;
    int rc;
    if (fused) {
        if ((rc = run_tv16(h, buckets, nbuckets, s, d_residuals))) return rc;
    } else {
        for (size_t i = 0; i < nbuckets; ++i) {
            const stg_bucket_t &b = buckets[i];
            if ((rc = run_device(h, b.key, b.d_src, b.d_src, b.n, b.k, b.d_idx, b.idx_cap, b.d_val, b.val_cap,
                                 b.idx_offset, b.d_count, s)))
                return rc;
        }
    }
    for (size_t i = 0; i < nbuckets; ++i)
        if (buckets[i].n && (rc = ef_after(h, buckets[i], d_residuals[i], fused, s))) return rc;
    return STG_OK;
}

int stg_codec_compress_wire_batch_device(stg_codec_t h, const stg_bucket_t *buckets, const int *flags,
                                         size_t nbuckets, void *stream) {
    CritPath crit_path;
    if (!h) return fail(STG_ERR_INVALID, "null codec handle");
    if (nbuckets && (!buckets || !flags)) return fail(STG_ERR_INVALID, "null bucket or flag array");
    if (h->method != M_TV16)
        return fail(STG_ERR_UNSUPPORTED, "wire-form emission is fused into thresholdv16 only "
                                         "(compress, then stg_wire_encode_device)");
    for (size_t i = 0; i < nbuckets; ++i) {
        const stg_bucket_t &b = buckets[i];
        const int rc = validate(h, b.n, b.k, b.idx_cap, b.val_cap, b.d_count);
        if (rc) return rc;
        if (flags[i] & ~3) return fail(STG_ERR_INVALID, "unknown wire flag bits");
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    // One bucket of 16-64 MiB: the one-bucket launch with its in-scan finish
    // (tv16lf2.h, which has no wire instance) into the workspace's staging,
    // then the separate packing -- 30.9 against 35.5 us fused for 64 MiB fp16
    // (profiles/r05_bench_configs_end.jsonl).
    if (nbuckets == 1 && flags[0] && buckets[0].n >= (size_t(1) << 22) &&
        buckets[0].n <= (size_t(1) << 24)) {
        const stg_bucket_t &b = buckets[0];
        HIP_TRY(hipSetDevice(h->device));
        Workspace *ws = nullptr;
        int rc = h->workspace(s, &ws);
        if (rc) return rc;
        stg_bucket_t t = b;
        // staging of its own, held for the whole sequence: another thread on
        // this stream cannot grow (free) it between the compress and the packing
        std::lock_guard<std::mutex> g(ws->wire_mu);
        if ((rc = ws->ensure_wire_stage(std::max<size_t>(b.idx_cap, 1)))) return rc;
        t.d_idx = ws->wst_pos;
        t.d_val = ws->wst_val;
        t.val_cap = t.idx_cap;
        if ((rc = run_tv16(h, &t, 1, s))) return rc;
        const size_t numel = std::min<size_t>(b.idx_cap, b.n);  // the pairs the fill writes
        HIP_TRY(stg::launch_wire_encode(t.d_idx, t.d_val, numel, (uint32_t)flags[0], b.d_idx, b.d_val, h->num_cu, s));
        return STG_OK;
    }
    return run_tv16(h, buckets, nbuckets, s, nullptr, nullptr, flags);
}

int stg_merge_gather_compress_device(stg_codec_t h, const stg_bucket_t *bucket, float *d_residual,
                                     const float *const *d_grads, int num_gpus, void *stream) {
    if (!h || !bucket) return fail(STG_ERR_INVALID, "null codec or bucket");
    if (num_gpus < 1 || num_gpus > (int)stg::GATHER_MAX) return fail(STG_ERR_INVALID, "num_gpus must be in [1, 16]");
    if (num_gpus > 1 && !d_grads) return fail(STG_ERR_INVALID, "null d_grads");
    for (int i = 1; i < num_gpus; ++i)
        if (bucket->n && !d_grads[i]) return fail(STG_ERR_INVALID, "null source");
    const stg_bucket_t &b = *bucket;
    int rc = validate(h, b.n, b.k, b.idx_cap, b.val_cap, b.d_count);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    HIP_TRY(hipSetDevice(h->device));
    stg::GatherArgs g{};
    g.dst = const_cast<float *>(b.d_src);
    g.resid = d_residual;
    g.nsrc = (uint32_t)num_gpus;
    for (int i = 1; i < num_gpus; ++i) g.src[i] = d_grads[i];
    if (h->method == M_TV16 && b.n) {
        float *res[1] = {d_residual};
        if ((rc = run_tv16(h, &b, 1, s, d_residual ? res : nullptr, &g))) return rc;
        return d_residual ? ef_after(h, b, d_residual, true, s) : STG_OK;
    }
    // the other codecs: the gather-add pass, then the task as without it
    HIP_TRY(stg::launch_gather_add(g, 0, b.n, h->num_cu, s));
    if (d_residual) return stg_merge_compress_batch_device(h, &b, &d_residual, 1, stream);
    return run_device(h, b.key, b.d_src, b.d_src, b.n, b.k, b.d_idx, b.idx_cap, b.d_val, b.val_cap, b.idx_offset,
                      b.d_count, s);
}

int stg_codec_compress_host(stg_codec_t h, const char *key, const float *src, size_t n, uint32_t k,
                            uint32_t *dst_idx, size_t idx_cap, float *dst_val, size_t val_cap, int32_t idx_offset,
                            size_t *out_count) {
    CritPath crit_path;
    if (!h || !out_count) return fail(STG_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s;
    int rc = thread_stream(h->device, &s);
    if (rc) return rc;
    Workspace *ws = nullptr;
    if ((rc = h->workspace(s, &ws))) return rc;
    {
        std::lock_guard<std::mutex> g(ws->mu);
        if ((rc = ws->grow(ws->h_src, ws->cap_src, std::max<size_t>(n, 1)))) return rc;
        size_t co = ws->cap_out;
        if ((rc = ws->grow(ws->h_idx, co, std::max<size_t>(idx_cap, 1)))) return rc;
        co = ws->cap_out;
        if ((rc = ws->grow(ws->h_val, co, std::max<size_t>(idx_cap, 1)))) return rc;
        ws->cap_out = co;
        if (!ws->h_count) HIP_TRY(hipMalloc(&ws->h_count, sizeof(uint32_t)));
        if (!ws->pinned_count) HIP_TRY(hipHostMalloc(&ws->pinned_count, 2 * sizeof(uint32_t)));
        if (n) HIP_TRY(hipMemcpyAsync(ws->h_src, src, n * sizeof(float), hipMemcpyHostToDevice, s));
    }
    // threshold-v keys its state by the caller's (host) src pointer
    rc = run_device(h, key, ws->h_src, src, n, k, ws->h_idx, idx_cap, ws->h_val, idx_cap, idx_offset, ws->h_count, s);
    if (rc) return rc;
    std::lock_guard<std::mutex> g(ws->mu);
    HIP_TRY(hipMemcpyAsync(ws->pinned_count, ws->h_count, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    if (idx_cap) {
        HIP_TRY(hipMemcpyAsync(dst_idx, ws->h_idx, idx_cap * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(dst_val, ws->h_val, std::min(idx_cap, val_cap) * sizeof(float), hipMemcpyDeviceToHost, s));
    }
    // the workspace's sticky failure word rides along: a device-side failure
    // (a bounded wait that gave up) is an error, never a silent wrong result
    HIP_TRY(hipMemcpyAsync(ws->pinned_count + 1, ws->d.fail, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (ws->pinned_count[1]) {
        char b[96];
        snprintf(b, sizeof b, "device failure flags 0x%x (details: stg_codec_check)", ws->pinned_count[1]);
        return fail(STG_ERR_DEVICE, b);
    }
    *out_count = *ws->pinned_count;
    return STG_OK;
}

int stg_codec_get_state(stg_codec_t h, const char *key, const void *key_ptr, float *threshold, float *threshold_inc,
                        void *stream) {
    if (!h) return fail(STG_ERR_INVALID, "null codec handle");
    HIP_TRY(hipSetDevice(h->device));
    KeyState *st = nullptr;
    {
        std::lock_guard<std::mutex> g(h->mu);
        auto it = h->slot_of.find(state_key(h->method, key, key_ptr));
        if (it == h->slot_of.end()) return fail(STG_ERR_INVALID, "key has no state yet");
        st = h->slot_ptr(it->second);
    }
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    KeyState hs;
    HIP_TRY(hipMemcpy(&hs, st, sizeof hs, hipMemcpyDeviceToHost));
    if (threshold) *threshold = hs.t;
    if (threshold_inc) *threshold_inc = hs.inc;
    return STG_OK;
}

int stg_codec_set_timing(stg_codec_t h, int enable) {
    if (!h) return fail(STG_ERR_INVALID, "null codec handle");
    std::lock_guard<std::mutex> g(h->mu);
    h->timing = enable != 0;
    return STG_OK;
}

int stg_codec_get_timing(stg_codec_t h, double *ms3, uint64_t *calls) {
    if (!h || !ms3 || !calls) return fail(STG_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(h->device));
    std::lock_guard<std::mutex> g(h->mu);
    for (auto &e : h->ev_pending) {
        HIP_TRY(hipEventSynchronize(e[2]));
        float a = 0, b = 0, c = 0;
        HIP_TRY(hipEventElapsedTime(&a, e[0], e[1]));
        HIP_TRY(hipEventElapsedTime(&b, e[1], e[2]));
        HIP_TRY(hipEventElapsedTime(&c, e[0], e[2]));
        h->ms_acc[0] += a;
        h->ms_acc[1] += b;
        h->ms_acc[2] += c;
        h->timed_calls++;
        h->ev_pool.push_back(e);
    }
    h->ev_pending.clear();
    for (int i = 0; i < 3; ++i) { ms3[i] = h->ms_acc[i]; h->ms_acc[i] = 0; }
    *calls = h->timed_calls;
    h->timed_calls = 0;
    return STG_OK;
}

int stg_codec_check(stg_codec_t h) {
    if (!h) return fail(STG_ERR_INVALID, "null codec handle");
    HIP_TRY(hipSetDevice(h->device));
    std::lock_guard<std::mutex> g(h->mu);
    for (auto &kv : h->ws) {
        HIP_TRY(hipStreamSynchronize(kv.first));
        uint32_t f[48] = {};
        HIP_TRY(hipMemcpy(f, kv.second->d.fail, sizeof f, hipMemcpyDeviceToHost));
        if (f[0]) {
            std::string m = "device failure flags 0x";
            char b[160];
            snprintf(b, sizeof b, "%x", f[0]);
            m += b;
            if (f[1]) {  // spin-timeout records (tv16.hip Ctx::spin_fail)
                snprintf(b, sizeof b, " (first spin timeout: site %u, workgroup %u, %u %u %u, epoch %u)", f[1] - 1, f[2],
                         f[3], f[4], f[5], f[6]);
                m += b;
                for (uint32_t site = 0; site < 10; ++site) {
                    const uint32_t *r = f + 8 + 4 * site;
                    if (!r[0]) continue;
                    snprintf(b, sizeof b, " [site %u: wg %u, %u %u %u]", site, r[0] - 1, r[1], r[2], r[3]);
                    m += b;
                }
            }
            return fail(STG_ERR_DEVICE, m);
        }
    }
    return STG_OK;
}

int stg_codec_debug_words(stg_codec_t h, void *stream, uint32_t *out, int n) {
    if (!h || !out || n < 0 || n > 64) return fail(STG_ERR_INVALID, "bad argument");
    HIP_TRY(hipSetDevice(h->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    Workspace *ws = nullptr;
    int rc = h->workspace(s, &ws);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    HIP_TRY(hipMemcpy(out, ws->d.misc, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return STG_OK;
}

int stg_error_feedback_device(float *d_grad, size_t n, const uint32_t *d_idx, size_t numel, float *d_residual,
                              void *stream) {
    if ((n && (!d_grad || !d_residual)) || (numel && !d_idx)) return fail(STG_ERR_INVALID, "null argument");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    int ncu = 256;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_TRY(stg::launch_error_feedback(d_grad, n, d_idx, numel, d_residual, ncu, static_cast<hipStream_t>(stream)));
    return STG_OK;
}

int stg_scatter_merge_device(const uint32_t *d_idx, const float *d_val, size_t per_rank, int world, size_t n,
                             float *d_dense, uint8_t *d_mark, uint32_t *d_out_idx, float *d_out_val,
                             uint32_t *d_out_count, void *stream) {
    if (world < 1) return fail(STG_ERR_INVALID, "world must be >= 1");
    if (world > 1 && (!d_dense || !d_mark)) return fail(STG_ERR_INVALID, "dense/mark scratch required for world > 1");
    if (world > 1 && (reinterpret_cast<uintptr_t>(d_mark) & 15u)) return fail(STG_ERR_INVALID, "mark scratch must be 16-byte aligned");
    if (n >= (size_t(1) << 32) || per_rank >= (size_t(1) << 32))
        return fail(STG_ERR_UNSUPPORTED, "more than 2^32-1 elements (uint32 indices)");
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    int ncu = 256;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    hipStream_t s = static_cast<hipStream_t>(stream);
    const std::shared_ptr<MergeScratch> ms = merge_scratch(dev, s);
    std::lock_guard<std::mutex> g(ms->mu);
    int rc = merge_scratch_ensure(ms.get(), s, n, per_rank, world);
    if (rc) return rc;
    if (++ms->tag == 0) ms->tag = 1;
    uint32_t grid = 0;
    const stg::Win1Desc w1{ms->desc, ms->ticket, 0, ms->tag, &grid, ms->fail,
                           reinterpret_cast<uint32_t *>(ms->ticket + 1)};
    HIP_TRY(stg::launch_scatter_merge(d_idx, d_val, per_rank, world, n, d_dense, d_mark, d_out_idx, d_out_val,
                                      d_out_count, ms->tiles, ms->win, ncu, s, w1));
    return STG_OK;
}

int stg_scatter_merge_check(void *stream) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    hipStream_t s = static_cast<hipStream_t>(stream);
    std::shared_ptr<MergeScratch> ms;
    {
        std::lock_guard<std::mutex> g(g_merge_mu);
        auto it = g_merge.find({dev, s});
        if (it == g_merge.end()) return STG_OK;  // no merge on this stream yet
        ms = it->second;
    }
    std::lock_guard<std::mutex> g(ms->mu);
    HIP_TRY(hipStreamSynchronize(s));
    uint32_t f = 0;
    if (ms->fail) HIP_TRY(hipMemcpy(&f, ms->fail, sizeof f, hipMemcpyDeviceToHost));
    if (f) {
        char b[96];
        snprintf(b, sizeof b, "MERGE decompress device failure flags 0x%x (a look-back gave up)", f);
        return fail(STG_ERR_DEVICE, b);
    }
    return STG_OK;
}

int stg_scatter_merge_release(void *stream) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    hipStream_t s = static_cast<hipStream_t>(stream);
    std::shared_ptr<MergeScratch> ms;
    {
        std::lock_guard<std::mutex> g(g_merge_mu);
        auto it = g_merge.find({dev, s});
        if (it == g_merge.end()) return STG_OK;
        ms = std::move(it->second);
        g_merge.erase(it);
    }
    {
        std::lock_guard<std::mutex> g(ms->mu);  // calls already inside finish first
        HIP_TRY(hipStreamSynchronize(s));
    }
    ms.reset();  // freed here, or by the last caller still holding it
    return STG_OK;
}

int stg_sgd_create(int device, float lr, float momentum, float dampening, float weight_decay, int nesterov,
                   int maximize, stg_sgd_t *out) {
    if (!out) return fail(STG_ERR_INVALID, "null argument");
    auto o = std::make_unique<stg_sgd>();
    o->device = device;
    o->lr = lr;
    o->momentum = momentum;
    o->dampening = dampening;
    o->weight_decay = weight_decay;
    o->nesterov = nesterov != 0;
    o->maximize = maximize != 0;
    *out = o.release();
    return STG_OK;
}

int stg_sgd_destroy(stg_sgd_t o) {
    delete o;
    return STG_OK;
}

// One optimize_raw call's launch arguments (the momentum buffer of `name`,
// created zeroed on its first call: sgd.cpp:40-47; the iteration count).
static int sgd_prepare(stg_sgd_t o, const char *name, float *d_param, uint32_t param_len, hipStream_t s,
                       stg::SgdLaunch *out) {
    bool first = false;
    float *mom = nullptr;
    {
        std::lock_guard<std::mutex> g(o->mu);
        if (o->momentum != 0.f) {
            auto it = o->mom.find(name);
            if (it == o->mom.end()) {  // sgd.cpp:40-47: zeroed buffer, first = true
                float *b = nullptr;
                HIP_TRY(hipMalloc(&b, std::max<size_t>(param_len, 1) * sizeof(float)));
                HIP_TRY(hipMemsetAsync(b, 0, std::max<size_t>(param_len, 1) * sizeof(float), s));
                o->mom.emplace(name, std::make_pair(b, param_len));
                mom = b;
                first = true;
            } else {
                mom = it->second.first;
            }
        }
        o->iter++;  // sgd.cpp:262
    }
    stg::SgdLaunch a{};
    a.param = d_param;
    a.param_len = param_len;
    a.mom = mom;
    a.first = first;
    a.momentum = o->momentum;
    a.dampening = o->dampening;
    a.weight_decay = o->weight_decay;
    a.lr = o->maximize ? -(double)o->lr : (double)o->lr;  // sgd.cpp:51
    a.nesterov = o->nesterov;
    *out = a;
    return STG_OK;
}

int stg_sgd_optimize_raw_device(stg_sgd_t o, const char *name, float *d_param, uint32_t param_len, const float *d_grad,
                                const uint32_t *d_idx, uint32_t grad_len, const uint32_t *d_grad_len, void *stream) {
    if (!o || !name) return fail(STG_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(o->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    stg::SgdLaunch a;
    int rc = sgd_prepare(o, name, d_param, param_len, s, &a);
    if (rc) return rc;
    a.grad = d_grad;
    a.gidx = d_idx;
    a.grad_len = grad_len;
    a.d_grad_len = d_grad_len;
    if (grad_len) HIP_TRY(stg::launch_sgd(a, s));
    return STG_OK;
}

int stg_merge_optimize_sgd_device(stg_sgd_t o, const char *name, float *d_param, uint32_t param_len,
                                  const uint32_t *d_idx, const float *d_val, size_t per_rank, int world,
                                  float *d_dense, uint8_t *d_mark, uint32_t *d_out_idx, float *d_out_val,
                                  uint32_t *d_out_count, void *stream) {
    if (!o || !name) return fail(STG_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(o->device));
    if (world != 1 || per_rank == 0) {  // the merge of several ranks, then the step over its output
        int rc = stg_scatter_merge_device(d_idx, d_val, per_rank, world, param_len, d_dense, d_mark, d_out_idx,
                                          d_out_val, d_out_count, stream);
        if (rc) return rc;
        const size_t cap = per_rank * (size_t)world;
        return stg_sgd_optimize_raw_device(o, name, d_param, param_len, d_out_val, d_out_idx,
                                           (uint32_t)std::min<size_t>(cap, 0xffffffffu), d_out_count, stream);
    }
    // world 1: the election, then the emission with every winner's step in the
    // same pass (each index is elected once, so the updates commute)
    if (per_rank >= (size_t(1) << 32) || param_len == 0)
        return fail(STG_ERR_UNSUPPORTED, "more than 2^32-1 elements or an empty parameter");
    hipStream_t s = static_cast<hipStream_t>(stream);
    stg::SgdLaunch a;
    int rc = sgd_prepare(o, name, d_param, param_len, s, &a);
    if (rc) return rc;
    int ncu = 256;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, o->device));
    const std::shared_ptr<MergeScratch> ms = merge_scratch(o->device, s);
    std::lock_guard<std::mutex> g(ms->mu);
    if ((rc = merge_scratch_ensure(ms.get(), s, param_len, per_rank, world))) return rc;
    if (++ms->tag == 0) ms->tag = 1;
    uint32_t grid = 0;
    stg::Win1Desc w1{ms->desc, ms->ticket, 0, ms->tag, &grid, ms->fail, reinterpret_cast<uint32_t *>(ms->ticket + 1)};
    w1.sgd = &a;
    HIP_TRY(stg::launch_scatter_merge(d_idx, d_val, per_rank, world, param_len, d_dense, d_mark, d_out_idx, d_out_val,
                                      d_out_count, ms->tiles, ms->win, ncu, s, w1));
    return STG_OK;
}

int stg_sgd_get_momentum(stg_sgd_t o, const char *name, float *host_out, uint32_t len, void *stream) {
    if (!o || !name) return fail(STG_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(o->device));
    float *b = nullptr;
    uint32_t n = 0;
    {
        std::lock_guard<std::mutex> g(o->mu);
        auto it = o->mom.find(name);
        if (it == o->mom.end()) return fail(STG_ERR_INVALID, "no momentum buffer for this name");
        b = it->second.first;
        n = it->second.second;
    }
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    HIP_TRY(hipMemcpy(host_out, b, std::min(len, n) * sizeof(float), hipMemcpyDeviceToHost));
    return STG_OK;
}

int stg_adam_create(int device, float lr, float b1, float b2, float eps, float weight_decay, int amsgrad,
                    int maximize, stg_adam_t *out) {
    if (!out) return fail(STG_ERR_INVALID, "null argument");
    auto o = std::make_unique<stg_adam>();
    o->device = device;
    o->lr = lr;
    o->b1 = b1;
    o->b2 = b2;
    o->eps = eps;
    o->weight_decay = weight_decay;
    o->amsgrad = amsgrad != 0;
    o->maximize = maximize != 0;
    *out = o.release();
    return STG_OK;
}

int stg_adam_destroy(stg_adam_t o) {
    delete o;
    return STG_OK;
}

// One optimize_raw call's launch arguments: the name's state (created zeroed
// on its first call: adam.cpp:28-35), its tick and the bias corrections.
static int adam_prepare(stg_adam_t o, const char *name, float *d_param, uint32_t param_len, hipStream_t s,
                        stg::AdamLaunch *out) {
    stg::AdamLaunch a{};
    uint32_t tick;
    {
        std::lock_guard<std::mutex> g(o->mu);
        if (!o->fail) {  // the handle's failure word, allocated with its first state
            HIP_TRY(hipMalloc(&o->fail, sizeof(uint32_t)));
            HIP_TRY(hipMemsetAsync(o->fail, 0, sizeof(uint32_t), s));
        }
        auto it = o->st.find(name);
        if (it == o->st.end()) {  // adam.cpp:28-35: zeroed m and v, vmax 0, tick 1
            stg_adam::Name nm;
            const size_t L = std::max<size_t>(param_len, 1);
            // one allocation: m | v | vmax
            HIP_TRY(hipMalloc(&nm.m, (2 * L + 1) * sizeof(float)));
            HIP_TRY(hipMemsetAsync(nm.m, 0, (2 * L + 1) * sizeof(float), s));
            nm.v = nm.m + L;
            nm.vmax = nm.m + 2 * L;
            if (o->amsgrad) {  // one tagged uint64 per tile; zero never matches a tick (>= 1)
                const size_t nt = (L + stg::ADAM_TILE - 1) / stg::ADAM_TILE;
                HIP_TRY(hipMalloc(&nm.tiles, nt * sizeof(uint64_t)));
                HIP_TRY(hipMemsetAsync(nm.tiles, 0, nt * sizeof(uint64_t), s));
            }
            nm.len = param_len;
            it = o->st.emplace(name, nm).first;
        }
        if (it->second.len != param_len) return fail(STG_ERR_INVALID, "param_len differs from the name's first call");
        a.m = it->second.m;
        a.v = it->second.v;
        a.vmax = it->second.vmax;
        a.tiles = it->second.tiles;
        tick = it->second.tick++;  // adam.cpp:40,82
    }
    a.param = d_param;
    a.param_len = param_len;
    a.b1 = o->b1;
    a.b2 = o->b2;
    a.eps = o->eps;
    a.weight_decay = o->weight_decay;
    a.lr = (double)o->lr;
    a.c1 = 1.0 - std::pow((double)o->b1, (double)tick);  // adam.cpp:42,67
    a.c2 = 1.0 - std::pow((double)o->b2, (double)tick);  // adam.cpp:43,68
    a.amsgrad = o->amsgrad;
    a.maximize = o->maximize;
    a.tag = tick;
    a.fail = o->fail;
    *out = a;
    return STG_OK;
}

int stg_adam_optimize_raw_device(stg_adam_t o, const char *name, float *d_param, uint32_t param_len,
                                 const float *d_grad, const uint32_t *d_idx, uint32_t grad_len,
                                 const uint32_t *d_grad_len, void *stream) {
    if (!o || !name) return fail(STG_ERR_INVALID, "null argument");
    if (o->amsgrad && grad_len > param_len)
        return fail(STG_ERR_INVALID, "amsgrad: grad_len > param_len (indices must be unique)");
    HIP_TRY(hipSetDevice(o->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    stg::AdamLaunch a;
    int rc = adam_prepare(o, name, d_param, param_len, s, &a);
    if (rc) return rc;
    a.grad = d_grad;
    a.gidx = d_idx;
    a.grad_len = grad_len;
    a.d_grad_len = d_grad_len;
    if (grad_len) HIP_TRY(stg::launch_adam(a, s));
    return STG_OK;
}

int stg_merge_optimize_adam_device(stg_adam_t o, const char *name, float *d_param, uint32_t param_len,
                                   const uint32_t *d_idx, const float *d_val, size_t per_rank, int world,
                                   float *d_dense, uint8_t *d_mark, uint32_t *d_out_idx, float *d_out_val,
                                   uint32_t *d_out_count, void *stream) {
    if (!o || !name) return fail(STG_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(o->device));
    if (world != 1 || per_rank == 0 || o->amsgrad) {  // the merge, then the step over its output
        int rc = stg_scatter_merge_device(d_idx, d_val, per_rank, world, param_len, d_dense, d_mark, d_out_idx,
                                          d_out_val, d_out_count, stream);
        if (rc) return rc;
        const size_t cap = std::min<size_t>(per_rank * (size_t)world, o->amsgrad ? param_len : 0xffffffffu);
        return stg_adam_optimize_raw_device(o, name, d_param, param_len, d_out_val, d_out_idx, (uint32_t)cap,
                                            d_out_count, stream);
    }
    // world 1 without amsgrad: the step inside the emission (see the SGD form)
    if (per_rank >= (size_t(1) << 32) || param_len == 0)
        return fail(STG_ERR_UNSUPPORTED, "more than 2^32-1 elements or an empty parameter");
    hipStream_t s = static_cast<hipStream_t>(stream);
    stg::AdamLaunch a;
    int rc = adam_prepare(o, name, d_param, param_len, s, &a);
    if (rc) return rc;
    int ncu = 256;
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, o->device));
    const std::shared_ptr<MergeScratch> ms = merge_scratch(o->device, s);
    std::lock_guard<std::mutex> g(ms->mu);
    if ((rc = merge_scratch_ensure(ms.get(), s, param_len, per_rank, world))) return rc;
    if (++ms->tag == 0) ms->tag = 1;
    uint32_t grid = 0;
    stg::Win1Desc w1{ms->desc, ms->ticket, 0, ms->tag, &grid, ms->fail, reinterpret_cast<uint32_t *>(ms->ticket + 1)};
    w1.adam = &a;
    HIP_TRY(stg::launch_scatter_merge(d_idx, d_val, per_rank, world, param_len, d_dense, d_mark, d_out_idx, d_out_val,
                                      d_out_count, ms->tiles, ms->win, ncu, s, w1));
    return STG_OK;
}

int stg_adam_get_state(stg_adam_t o, const char *name, float *host_m, float *host_v, uint32_t len,
                       float *host_vmax, uint32_t *tick_out, void *stream) {
    if (!o || !name) return fail(STG_ERR_INVALID, "null argument");
    stg_adam::Name nm;
    {
        std::lock_guard<std::mutex> g(o->mu);
        auto it = o->st.find(name);
        if (it == o->st.end()) return fail(STG_ERR_INVALID, "no Adam state for this name");
        nm = it->second;
    }
    HIP_TRY(hipSetDevice(o->device));
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    const size_t c = std::min(len, nm.len);
    if (host_m) HIP_TRY(hipMemcpy(host_m, nm.m, c * sizeof(float), hipMemcpyDeviceToHost));
    if (host_v) HIP_TRY(hipMemcpy(host_v, nm.v, c * sizeof(float), hipMemcpyDeviceToHost));
    if (host_vmax) HIP_TRY(hipMemcpy(host_vmax, nm.vmax, sizeof(float), hipMemcpyDeviceToHost));
    if (tick_out) *tick_out = nm.tick;
    return STG_OK;
}

int stg_adam_check(stg_adam_t o, void *stream) {
    if (!o) return fail(STG_ERR_INVALID, "null argument");
    HIP_TRY(hipSetDevice(o->device));
    HIP_TRY(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    uint32_t f = 0;
    if (o->fail) HIP_TRY(hipMemcpy(&f, o->fail, sizeof f, hipMemcpyDeviceToHost));
    if (f) return fail(STG_ERR_DEVICE, "adam: amsgrad look-back timed out (a predecessor tile never published)");
    return STG_OK;
}

int stg_gather_slice(uint64_t n, int local_rank, int num_gpus, uint64_t *start, uint64_t *end) {
    if (!start || !end) return fail(STG_ERR_INVALID, "null argument");
    if (num_gpus < 1 || local_rank < 0 || local_rank >= num_gpus) return fail(STG_ERR_INVALID, "bad rank / GPU count");
    *start = (uint64_t)(((int64_t)n * local_rank) / num_gpus);  // cpu_gather.cpp:59-60 (int64 arithmetic)
    *end = (uint64_t)(((int64_t)n * (local_rank + 1)) / num_gpus);
    return STG_OK;
}

int stg_gather_add_device(float *d_grad0, const float *d_residual, const float *const *d_grads, int num_gpus,
                          uint64_t n, int local_rank, void *stream) {
    if (num_gpus < 1 || num_gpus > (int)stg::GATHER_MAX) return fail(STG_ERR_UNSUPPORTED, "num_gpus outside 1..16");
    uint64_t a = 0, b = 0;
    int rc = stg_gather_slice(n, local_rank, num_gpus, &a, &b);
    if (rc) return rc;
    if (a == b) return STG_OK;
    if (!d_grad0 || (num_gpus > 1 && !d_grads)) return fail(STG_ERR_INVALID, "null argument");
    stg::GatherArgs g{};
    g.dst = d_grad0;
    g.resid = d_residual;
    g.nsrc = (uint32_t)num_gpus;
    for (int i = 1; i < num_gpus; ++i) {
        if (!d_grads[i]) return fail(STG_ERR_INVALID, "null source");
        g.src[i] = d_grads[i];
    }
    int dev = 0, ncu = 256;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_TRY(stg::launch_gather_add(g, a, b, ncu, static_cast<hipStream_t>(stream)));
    return STG_OK;
}

int stg_wire_flag(uint64_t tensor_numel, int fp16_values) {
    return (tensor_numel < 65536 ? STG_WIRE_U16_IDX : 0) | (fp16_values ? STG_WIRE_F16_VAL : 0);
}

int stg_wire_encode_device(const uint32_t *d_idx, const float *d_val, size_t numel, int flag, void *d_idx_out,
                           void *d_val_out, void *stream) {
    if (flag & ~(STG_WIRE_U16_IDX | STG_WIRE_F16_VAL)) return fail(STG_ERR_INVALID, "unknown wire flag bits");
    if (!numel) return STG_OK;
    if (!d_idx || !d_val || !d_idx_out || !d_val_out) return fail(STG_ERR_INVALID, "null argument");
    int dev = 0, ncu = 256;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_TRY(stg::launch_wire_encode(d_idx, d_val, numel, (uint32_t)flag, d_idx_out, d_val_out, ncu,
                                    static_cast<hipStream_t>(stream)));
    return STG_OK;
}

int stg_wire_encode_batch_device(const stg_wire_stream_t *streams, size_t nstreams, void *stream) {
    if (nstreams && !streams) return fail(STG_ERR_INVALID, "null stream array");
    for (size_t i = 0; i < nstreams; ++i) {
        const stg_wire_stream_t &w = streams[i];
        if (w.flag & ~(STG_WIRE_U16_IDX | STG_WIRE_F16_VAL)) return fail(STG_ERR_INVALID, "unknown wire flag bits");
        if (w.numel && (!w.d_idx || !w.d_val || !w.d_idx_out || !w.d_val_out))
            return fail(STG_ERR_INVALID, "null argument");
        if (w.numel > (size_t)STG_WG * 0xffffffull) return fail(STG_ERR_UNSUPPORTED, "wire stream too long for a batch");
    }
    hipStream_t s = static_cast<hipStream_t>(stream);
    stg::WireBatch b{};
    uint64_t blocks = 0;
    auto flush = [&]() -> int {
        if (b.nb) HIP_TRY(stg::launch_wire_encode_batch(b, (uint32_t)blocks, s));
        b = stg::WireBatch{};
        blocks = 0;
        return STG_OK;
    };
    for (size_t i = 0; i < nstreams; ++i) {
        const stg_wire_stream_t &w = streams[i];
        if (!w.numel) continue;
        const uint64_t nbk = (w.numel + STG_WG - 1) / STG_WG;
        if (b.nb == stg::WIRE_BATCH || blocks + nbk > 0x7fffffffull) {
            int rc = flush();
            if (rc) return rc;
        }
        stg::WireBucket &d = b.b[b.nb++];
        d.idx = w.d_idx;
        d.val = w.d_val;
        d.idx_out = w.d_idx_out;
        d.val_out = w.d_val_out;
        d.n = w.numel;
        d.flag = (uint32_t)w.flag;
        d.blk0 = (uint32_t)blocks;
        blocks += nbk;
    }
    return flush();
}

int stg_wire_decode_device(const void *d_idx_in, const void *d_val_in, size_t numel, int flag, uint32_t *d_idx,
                           float *d_val, void *stream) {
    if (flag & ~(STG_WIRE_U16_IDX | STG_WIRE_F16_VAL)) return fail(STG_ERR_INVALID, "unknown wire flag bits");
    if (!numel) return STG_OK;
    if (!d_idx_in || !d_val_in || !d_idx || !d_val) return fail(STG_ERR_INVALID, "null argument");
    int dev = 0, ncu = 256;
    HIP_TRY(hipGetDevice(&dev));
    HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_TRY(stg::launch_wire_decode(d_idx_in, d_val_in, numel, (uint32_t)flag, d_idx, d_val, ncu,
                                    static_cast<hipStream_t>(stream)));
    return STG_OK;
}

int stg_synth_fill_device(float *d_dst, size_t n, uint64_t seed, int dist, uint32_t param, void *stream) {
    if (!n) return STG_OK;
    HIP_TRY(stg::launch_synth(d_dst, n, seed, dist, param, static_cast<hipStream_t>(stream)));
    return STG_OK;
}

}  // extern "C"
