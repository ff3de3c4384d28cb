// ws.h -- per-stream workspace layout shared by host launchers and kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace stg {

constexpr uint32_t CAND_CAP = 8192;          // regime-B window entries per bucket (+1 for the ragged tail)
constexpr uint32_t CAND_WORDS = 4 * CAND_CAP; // per bucket: line-sum bits | line position | candidate index | spare
constexpr uint32_t TV16_WIN = 1u << 18;      // regime-B window below t, in ulps of t (~3.1 %)
constexpr uint32_t TV16_SCAN_LDS = 35584;     // LDS bytes of a scan workgroup (bound; tv16.hip checks)

constexpr uint32_t TV_TILE = 8192;           // top-k elements per tile (32 KiB)
constexpr uint32_t TOPK_SUP_CAP = 1024;      // top-k superset entries kept per tile
constexpr uint32_t TOPK_LIST_CAP = 4096;     // top-k: keys of T's level-2 bin listed for the final select
constexpr uint32_t TOPK_LIST_TILES = 8192;   // ... when the bucket has at most this many tiles (64 Mi floats)
constexpr uint32_t TV_MAXG = 2048;           // threshold-v ranges (workgroups) per call
constexpr uint32_t TV_SCAP = 4096;           // threshold-v qualifiers listed per range (32 KiB of LDS)

constexpr uint32_t RS_BINS = 2048;           // radix-select bins (11 bits)
constexpr uint32_t RS_SHARDS = 8;            // histogram copies: workgroup w adds into shard w % RS_SHARDS
constexpr uint32_t RS_SH_HIST = 4;           // ... of which rs_hist's one workgroup per CU uses the first 4

// thresholdv16 in-launch control block (one launch = a batch of <= MAX_BATCH
// buckets cut into fixed 2048-line chunks).  The per-call chunk counter comes
// in two copies selected by the call epoch's parity; every launch zeroes the
// other copy for the next call (the next call on this workspace is
// stream-ordered after this launch).  Words handed between workgroups carry
// the call tag (epoch << 8 | kind) so stale words of earlier calls never match.
constexpr uint32_t MAX_BATCH = 32;
constexpr uint32_t TV16_CHUNK = 2048;        // lines (16 floats) per chunk = 128 KiB
struct CallCtl {
    uint32_t next;      // dynamic chunk counter
    uint32_t pad[31];
    uint32_t crew_ticket[32];  // the crew's ticket (its own line: taken by every crew workgroup)
    uint32_t crew_done[32];    // the crew's completed units per phase (polled)
};
// Per-bucket regime decision, written by the finisher of the bucket's last
// chunk: [1..3] first, drained, then [0] = {tag:32 | flags:32}; read by the
// follow-on fill launch.
struct alignas(32) Decision {
    uint64_t w[4];      // [1] = {cnt:32 | M:32}, [2] = {Wtot:32 | tail key bits:32}, [3] = {Qtot:32 | t bits:32}
};
constexpr uint32_t TV16_DEC_B = 1, TV16_DEC_WIN = 2, TV16_DEC_TAIL = 4;  // Decision flags
constexpr uint32_t TV16_TAG_DEC = 3;
constexpr uint32_t POISON_COUNT = 0xffffffffu;  // *count_out of a launch that hit a device failure
struct FillCtl {
    CallCtl cc[2];                     // [epoch parity]
    Decision dec[MAX_BATCH];
};
// Per-chunk descriptor (16 B): {tag:32 | qualifying lines:16 | window lines:16}
// by the chunk's last streaming wave.
struct alignas(16) ChunkDesc {
    uint64_t agg;
    uint64_t pad;
};

// Per-call scalars handed from the scan kernel to the fill kernel.
struct CallParams {
    float t;
    float inc;
    uint32_t pad[2];
};

// Radix-select state (first thresholds, top-k).
struct RSel {
    uint32_t prefix;    // bits fixed so far
    uint32_t mask;      // which bits are fixed
    uint32_t rank;      // remaining rank (0-based, descending) inside the prefix
    uint32_t cnt_gt;    // keys strictly above the prefix range
    uint32_t done;      // classes of workgroups done with the current pass (the last one picks)
    uint32_t pad[3];    // pad[0]: top-k's superset floor; [1]: keys in the last picked bin; [2]: top-k list length
    uint32_t done64[64];  // workgroups done, per class blockIdx.x % 64
    // The level histogram in RS_SHARDS copies, summed by the pick: device-scope
    // atomics on one word serialise at the memory side (~90 per us), so a
    // 2048-workgroup pass adding into one copy spent ~15 us on its hot bins
    // (into 8 copies: 256 adds per word, spread over the pass).
    uint32_t hist[RS_SHARDS][RS_BINS];
};

// thresholdv16 one-bucket path: a scan launch with no waits between
// workgroups (tv16_lscan, tv16lone.hip) lists, per chunk, its qualifying and
// window lines; the fill launch (tv16fill.hip, lfin mode) finishes the call.
constexpr uint32_t LCHUNK = 512;  // lines (16 floats) per chunk = 32 KiB: one per 256-thread workgroup
constexpr uint32_t LQCAP = 64;    // qualifying lines listed per chunk (~5 at k = 1 %; more: the finish re-reads it)
constexpr uint32_t LWCAP = 32;    // window lines listed per chunk (~2; more: likewise)
constexpr uint32_t LMAXC = 4096;  // chunks of a bucket the one-bucket path takes (128 MiB)
// ... and its window entries binned by the scan: bin b = (bits(t) - 1 - bits(sum)) >> 8
// (256 ulps, 1024 bins over the window), LBCAP entries per bin {sum bits,
// chunk << 19 | line within the chunk << 10 | qualifying lines before it};
// the counts are zeroed by the finish's last workgroup after use
constexpr uint32_t LNBIN = 1024;
constexpr uint32_t LBCAP = 32;
// bin b's count word: bins interleaved over 32 lines (b mod 32 picks the
// line), so the bins the window fills near t sit on as many 128-byte lines
// (the scan's returning atomics on one line queue behind each other)
__host__ __device__ constexpr uint32_t whist_word(uint32_t b) { return (b & 31u) * 32u + (b >> 5); }
static_assert(LNBIN == 1024, "32 lines x 32 words");

// thresholdv16 regime-B crew (tv16wide.h): per bucket slot of a launch, the
// level-1 histogram of the candidates' keys and the hand-offs between phases
constexpr uint32_t CREW_BINS = 8192;
struct CrewCtl {
    uint32_t hist[CREW_BINS];  // zeroed by the bucket's phase Z
    uint32_t beta, nL, status, P, tail_rank, op, pad[2];
};

// top-k steered by the key's last k-th magnitude (topk1.hip): per-call control
// block, two copies by call tag parity (each call zeroes the next call's), and
// the band histogram (one bin per ulp, two copies by parity)
constexpr uint32_t TK1_NPH = 9;     // phases of the select's way
constexpr uint32_t TK1_SH = 8;      // ticket / completion shards (tile % 8); superset regions
constexpr uint32_t TK1_LINE = 32;   // words per 128-byte line: every shard counter on a line of its own
constexpr uint32_t TK2_FINE = 1u << 18;               // band bins: one per ulp
constexpr uint32_t TK2_CSH = 8;                       // coarse bins: 256 ulps
constexpr uint32_t TK2_COARSE = TK2_FINE >> TK2_CSH;  // 1024
constexpr uint32_t kTk2Cshards = 1;  // 4 and 8 copies measured slower (profiles/r05_topk_finish_ab.jsonl)
constexpr uint32_t TK2_CSHARDS = kTk2Cshards;     // copies of the coarse bins (each tile adds into one)
constexpr uint32_t TK2_HI = 16;                       // shards of the count of keys above the band
constexpr uint32_t TK2_REG = 32;                      // superset regions (tile mod 32), an offset counter each
constexpr uint32_t kTk2Ut = 16;
constexpr uint32_t TK2_UT = kTk2Ut;               // tiles per emission unit (at most)
constexpr uint32_t TK2_UNITS = TOPK_LIST_TILES / TK2_UT;
struct alignas(128) TopkCtl {
    // the stream launch's band [F, H): the next call's stream launch zeroes
    // the fine bins [0, H - F) it touched and every line after this one
    uint32_t band_F, band_H, band_ok;
    uint32_t bpad[TK1_LINE - 3];
    uint32_t tk[TK1_NPH][TK1_SH][TK1_LINE];    // tickets per phase and shard
    uint32_t done[TK1_NPH][TK1_SH][TK1_LINE];  // units done per phase and shard
    uint32_t sdone[TK1_NPH][TK1_LINE];         // shards done per phase
    uint32_t flag[TK1_NPH];                    // = the call tag once single-unit phase p is done
    uint32_t ovf, res_T;                       // a superset region overflowed; the select's T
    uint32_t pad[TK1_LINE - TK1_NPH - 2];
    uint32_t utk[TK1_LINE];                    // emission units taken
    uint32_t hi[TK2_HI][TK1_LINE];             // keys >= H, by tile % TK2_HI
    uint32_t shn[TK2_REG][TK1_LINE];           // superset entries placed in region tile % TK2_REG
    uint32_t coarse[TK2_CSHARDS][TK2_COARSE];  // band keys per 256 ulps, by tile % TK2_CSHARDS
    uint64_t udesc[TK2_UNITS];                 // emission unit u: bit 63 | > T count << 32 | == T count
};

struct DevWS {
    FillCtl *ctl;
    TopkCtl *tkctl;      // [2]
    uint32_t *tkfine;    // [2][TK2_FINE] band histograms by call parity, zero between calls
    CrewCtl *crew;       // MAX_BATCH slots
    ChunkDesc *desc;     // thresholdv16 chunk descriptors (grown per launch, zeroed)
    CallParams *cp;
    RSel *rsel;
    uint32_t *fail;      // sticky failure bits
    uint32_t *cand;      // regime-B window entries, CAND_WORDS per bucket of a launch
    uint32_t *misc;      // small scratch (counts)
    uint64_t *tv_ticket;   // threshold-v: ranges taken, monotonic over the workspace's life
    float *sums;         // thresholdv16: one sum per 16-float line
    uint32_t *tile_cnt;  // per-tile qualifier counts
    uint32_t *tile_aux;  // per-tile secondary counts (threshold-v max, top-k ties)
    uint32_t *stage_pos; // threshold-v staged positions
    float *stage_val;    // threshold-v staged values
    uint2 *ldesc;        // one-bucket path: per chunk {qualifying lines, window lines}
    uint32_t *lq;        // ... the chunk's qualifying lines in order (LQCAP per chunk, line within the chunk)
    uint2 *lw;           // ... its window lines in order: {sum bits, line within the chunk | qualifying before << 16}
    float4 *lv;          // ... the qualifying lines' data (LQCAP x 4 float4 per chunk)
    uint32_t *whist;     // ... window entries per bin (2 x LNBIN by call parity, zero between calls)
    uint32_t *larr;      // ... the scan's finish: per role the tag of the last call it finished
    uint2 *went;         // ... the entries by bin (LNBIN x LBCAP)
};

// ---- launchers (implemented in the .hip files) ----
constexpr uint32_t GATHER_MAX = 16;  // local GPUs per node the gather-add accepts
struct GatherArgs {
    float *dst;                    // grad[0]
    const float *resid;            // residual (or null: no residual term)
    const float *src[GATHER_MAX];  // src[1 .. nsrc-1] = grad[1 .. N-1]; src[0] unused
    uint32_t nsrc;                 // N, the node's GPU count
};
struct Tv16Bucket {
    const float *src;
    size_t n;
    uint32_t k;
    uint32_t dst_len;
    uint32_t *idx;
    float *val;
    int32_t idx_offset;
    uint32_t *count_out;
    KeyState *state;
    bool first;        // no AIMD state yet: compute the first threshold
    float *sums;       // per-bucket scratch: first-threshold line sums; the fill's candidate heap
                       // (2 words per line: (nb + 1) * 2 floats)
    float *resid;      // MERGE error feedback: receives the bucket's full lines, or null
    const GatherArgs *gather;  // intra-node gather-add fused into the scan (dst = src), or null
    uint32_t wflag;    // the emission writes the wire form (STG_WIRE_* flags; idx / val typed by it)
};
struct Tv16Launch {
    const Tv16Bucket *b;
    uint32_t nb;       // buckets in this launch (<= MAX_BATCH)
    int num_cu;
    hipEvent_t *ev;    // optional [before, mid, after] the codec launch(es)
    uint32_t epoch;    // per-workspace call counter, 1..2^24-1 (hand-off tags)
    uint32_t max_wg;     // fused-kernel workgroups at most (its share of 2 per CU)
    uint32_t desc_cap;   // ChunkDesc entries at ws.desc
    uint32_t lone_cap;   // chunks the one-bucket lists (ws.ldesc / lq / lw) hold (0: none)
    uint32_t *lone_calls;  // the workspace's one-bucket path calls (host; its parity picks the
                           // window histogram and arrival block, each call zeroing the other copy)
};
hipError_t launch_tv16(const Tv16Launch &a, const DevWS &ws, hipStream_t s);
// thresholdv16 regime-B heap fill (tv16fill.hip): one workgroup per bucket
struct Tv16FillBucket {
    const float *src;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    uint32_t nb, tl, dst_len;
    int32_t idx_offset;
    const uint32_t *cand;  // the bucket's window entries (CAND_WORDS)
    uint2 *heap;           // full-path scratch: (nb + 1) candidates {key bits, element position}
    uint32_t wflag, wend;  // wire form of the emitted pairs (wire_dev.h; 0: u32 / f32)
};
struct Tv16FillArgs {
    Tv16FillBucket bk[MAX_BATCH];
    uint32_t nbk;
    uint32_t epoch;
    const Decision *dec;
    uint32_t *fail;
    uint32_t *dbg;         // diagnostics: phase stamps of workgroup 0 (ws.misc)
    uint32_t mode;         // tests (STG_DEBUG_TV16_FILL): 1 = always the shadow heap, 2 = always the literal heap,
                           // 3 = always the leader over the window, 4 = always the crew
    uint32_t crew;         // extra workgroups that order window-miss buckets (tv16wide.h; 0: none)
    CrewCtl *crew_ctl;     // MAX_BATCH slots
    bool lone;             // a one-bucket launch: the fill variant that takes the CU's registers
    uint32_t helpers;      // lone: extra workgroups that emit shares of the order (0: none)
    CallCtl *cc;           // this call's counters: [pad 0] fill tickets, [1] order ready, [2] pops, [3] tail rank,
                           // [4] lfin workers done
    // lfin: the launch also finishes a one-bucket scan (tv16_lscan): `workers`
    // workgroups emit the qualifying lines, list the window and decide; the
    // last of them to finish orders the regime-B fill; `helpers` more emit it
    bool lfin;
    uint32_t workers;
    uint32_t nc;           // chunks of the bucket
    const uint2 *ldesc;
    const uint32_t *lq;
    const uint2 *lw;
    const float4 *lv;
    uint32_t *whist;       // the scan's binned window (this call's copy; the scan zeroes the next call's)
    const uint2 *went;
    uint32_t rankers;      // workgroups that order the regime-B fill in parallel (0: the orderer alone)
    KeyState *state;
    const CallParams *cp;  // {t, inc} as the scan read them
    float *resid;          // fused error feedback: the ragged tail is copied by the finish
    // the scan launch finished the call (tv16lf2.h): every role of this launch
    // leaves when fin_done[0 .. fin) all hold fin_tag (fin == 0: never)
    const uint32_t *fin_done;
    uint32_t fin, fin_tag;
};
hipError_t launch_tv16_fill(const Tv16FillArgs &a, hipStream_t s);
// the same fill built to write the wire form of buckets with wflag set (tv16fill.hip)
hipError_t launch_tv16_fill_wire(const Tv16FillArgs &a, hipStream_t s);
inline hipError_t launch_tv16_fill_any(const Tv16FillArgs &a, hipStream_t s) {
    bool w = false;
    for (uint32_t i = 0; i < a.nbk; ++i) w |= a.bk[i].wflag != 0;
    return w ? launch_tv16_fill_wire(a, s) : launch_tv16_fill(a, s);
}
// one-bucket scan (tv16lone.hip): every workgroup streams its chunks and lists
// them; nothing waits on another workgroup
constexpr uint32_t LF2_MAXF = 64;                     // finish roles of a one-bucket scan at most (tv16lf2.h)
constexpr uint32_t LARR_WORDS = LF2_MAXF;             // per role: the call tag once its part is written
struct LScanArgs {
    const float *src;
    uint32_t nb;           // full lines
    uint32_t nc;           // chunks
    KeyState *state;
    CallParams *cp;        // receives {t, inc} as read
    float *resid;          // fused error feedback (or null)
    uint2 *ldesc;
    uint32_t *lq;
    uint2 *lw;
    float4 *lv;
    uint32_t *whist;       // window entries per bin (zero at the start of the call)
    uint2 *went;           // ... and the entries, LBCAP per bin
    uint32_t *zero_next;   // the next call's counter block (CallCtl), zeroed here
    // the gather-add fused into the stream (gather.hip's sum, in its order):
    // src += gres + gsrc[1] + ... + gsrc[gn - 1], stored back to src once
    const float *gres;     // residual term (null: none)
    const float *gsrc[GATHER_MAX];
    uint32_t gn;           // 0: no gather; else N (gsrc[0] unused)
    uint32_t tl;           // the ragged tail's floats (summed by workgroup 0 under the gather)
    // the finish inside the scan launch (tv16lf2.h): `fin` roles (0: none, the
    // fill launch finishes), `nwk` of them workers; arrival block of this call
    // and of the next (zeroed here), and the next call's window histogram
    uint32_t fin, nwk, mode;
    uint32_t tag;          // the call's tag (>= 1) on every chunk's counts
    uint32_t skip;         // diagnostics (STG_LF2_SKIP): a role stops at that point (5: the lists carry a wrong tag)
    uint32_t *done;        // per role: the tag once its part is written (LARR_WORDS)
    uint32_t *whist_next;
    uint32_t *out_idx;
    float *out_val;
    uint32_t *count_out;
    uint32_t dst_len;
    int32_t idx_offset;
    uint32_t *fail, *dbg;
};
hipError_t launch_tv16_lscan(LScanArgs &a, int num_cu, hipStream_t s);

struct TvLaunch {
    const float *src;
    size_t n;
    uint32_t k;
    uint32_t cap;
    uint32_t *idx;
    float *val;
    uint32_t *count_out;
    KeyState *state;
    bool first;
    int num_cu;
    hipEvent_t *ev;
    uint32_t tag;          // call tag (>= 1) of the range descriptors at ws.tile_cnt (2 words per range)
    uint64_t ticket_base;  // ws.tv_ticket's value when this call starts
    uint32_t *grid_out;    // receives the launch's range count (the ticket advances by it)
};
hipError_t launch_tv(const TvLaunch &a, const DevWS &ws, hipStream_t s);

struct TopkLaunch {
    const float *src;
    size_t n;
    uint32_t k;
    uint32_t cap;
    uint32_t *idx;
    float *val;
    int32_t idx_offset;
    bool bug_compat;
    uint32_t *count_out;
    int num_cu;
    hipEvent_t *ev;
};
hipError_t launch_topk(const TopkLaunch &a, const DevWS &ws, hipStream_t s);
// top-k steered by the key's last k-th magnitude (topk1.hip), buckets of at
// most TOPK_LIST_TILES tiles: a key's first call (!hinted) runs launch_topk and
// seeds the hint; later calls stream once and emit (the select's way inside
// the emission launch when the band misses)
hipError_t launch_topk1(const TopkLaunch &a, const DevWS &ws, KeyState *state, bool hinted, uint32_t *tag,
                        hipStream_t s);

// Radix select: the key of descending rank `rank` among (bits(a[i]) & 0x7fffffff),
// i < m, with the last element's bits additionally masked by `last_mask`, plus
// `extra_zeros` implicit zero keys.  Result in ws.rsel (prefix = key bits,
// cnt_gt = keys strictly greater, rank = rank among equal keys).
hipError_t launch_radix_select(const float *a, size_t m, uint32_t last_mask, uint64_t extra_zeros, uint32_t rank,
                               const DevWS &ws, int num_cu, hipStream_t s);
hipError_t launch_radix_level1(const float *a, size_t m, uint32_t last_mask, uint64_t extra_zeros, uint32_t rank,
                               const DevWS &ws, int num_cu, hipStream_t s);

hipError_t launch_synth(float *dst, size_t n, uint64_t seed, int dist, uint32_t param, hipStream_t s);

// world == 1 in one launch after the winner election: tagged per-tile counts
// and a ticket counter of the (device, stream) scratch (desc == nullptr: the
// two-launch count / emit instead)
struct Win1Desc {
    uint64_t *desc;       // per tile {tag:32 | winners:32}, zero at creation
    uint64_t *ticket;     // tile counter, zeroed by each call's win_mark
    uint64_t base;        // unused (0)
    uint32_t tag;         // call tag >= 1
    uint32_t *grid_out;   // receives the tiles launched (the ticket advances by it)
    uint32_t *fail;       // sticky failure word of the scratch (a look-back that gave up)
    uint32_t *dup;        // world 1: set when an index repeats; the ticket then counts from 0 (win_mark zeroes it)
    const struct SgdLaunch *sgd = nullptr;    // world 1: the SGD step fused into the emission (null: none)
    const struct AdamLaunch *adam = nullptr;  // ... or the Adam step (no amsgrad)
};
hipError_t launch_scatter_merge(const uint32_t *idx, const float *val, size_t per_rank, int world, size_t n,
                                float *dense, uint8_t *mark, uint32_t *out_idx, float *out_val,
                                uint32_t *out_count, uint32_t *scratch_tiles, uint32_t *win, int num_cu,
                                hipStream_t s, const Win1Desc &w1);
constexpr uint32_t MERGE_TILE = STG_WG * 16;  // pairs / marks per scatter-merge tile

struct SgdLaunch {
    float *param;
    uint32_t param_len;
    const float *grad;
    const uint32_t *gidx;
    uint32_t grad_len;
    const uint32_t *d_grad_len;
    float *mom;      // momentum buffer (param_len floats) or null when momentum == 0
    bool first;
    float momentum, dampening, weight_decay;
    double lr;
    bool nesterov;
};
hipError_t launch_sgd(const SgdLaunch &a, hipStream_t s);

struct AdamLaunch {
    float *param;
    uint32_t param_len;
    const float *grad;
    const uint32_t *gidx;
    uint32_t grad_len;          // capacity of grad/gidx (grid size)
    const uint32_t *d_grad_len; // device count (min'd with grad_len) or null
    float *m, *v;               // per-name moment arrays (param_len floats each)
    float *vmax;                // per-name running max (one float on the device)
    uint32_t *tiles;            // amsgrad look-back words: one uint64 per ADAM_TILE tile (zeroed at allocation)
    uint32_t tag;               // amsgrad word tag: the name's tick of this call (>= 1)
    uint32_t *fail;             // sticky device failure word of the optimizer handle
    float b1, b2, eps, weight_decay;
    double lr, c1, c2;          // c = 1 - pow(b, tick), computed on the host (adam.cpp:42-43,67-68)
    bool amsgrad, maximize;
};
constexpr uint32_t ADAM_TILE = STG_WG * 4;  // amsgrad: elements per workgroup tile
hipError_t launch_adam(const AdamLaunch &a, hipStream_t s);
hipError_t launch_gather_add(const GatherArgs &a, size_t start, size_t end, int num_cu, hipStream_t s);
constexpr uint32_t WIRE_BATCH = 16;  // buckets per batched wire launch
struct WireBucket {
    const uint32_t *idx;
    const float *val;
    void *idx_out, *val_out;
    uint64_t n;
    uint32_t flag, blk0;  // blk0: first workgroup of this bucket in the launch
};
struct WireBatch {
    WireBucket b[WIRE_BATCH];
    uint32_t nb;
};
hipError_t launch_wire_encode_batch(const WireBatch &w, uint32_t blocks, hipStream_t s);
hipError_t launch_wire_encode(const uint32_t *idx, const float *val, size_t n, uint32_t flag, void *idx_out,
                              void *val_out, int num_cu, hipStream_t s);
hipError_t launch_wire_decode(const void *idx_in, const void *val_in, size_t n, uint32_t flag, uint32_t *idx,
                              float *val, int num_cu, hipStream_t s);
hipError_t launch_ef_zero(float *grad, float *resid, const uint32_t *idx, size_t numel, size_t n, int num_cu,
                          hipStream_t s);
hipError_t launch_error_feedback(float *grad, size_t n, const uint32_t *idx, size_t numel, float *resid, int num_cu,
                                 hipStream_t s);

}  // namespace stg
