/*
 * stg/codec.h -- C-ABI of the MI355X-native StellaTrain gradient codec.
 *
 * This is the drop-in boundary.  It replaces the reference's
 *   class Compressor { virtual size_t compress(const std::string &name,
 *       ConstSegment<float> src, uint32_t k, Segment<uint32_t> dst_idx,
 *       Segment<float> dst_val, int32_t idx_offset = 0) = 0; }
 * (/root/reference/backend/src/compress/compressor.h:12-31) and its three
 * factory-selected implementations (engine/core.cpp:110-118, 185-195):
 *   "thresholdv16" -> ThresholdvCompressor16  (compress/thresholdv16.h:9-38)
 *   "thresholdv"   -> ThresholdvCompressor    (compress/thresholdv.h:9-29)
 *   "topk"         -> TopkCompressor          (compress/topk.h:9-31)
 * plus the inverse path of config 5: the MERGE decompress
 * (engine/modules/cpu_optimize.cpp:40-72) and the sparse SGD apply
 * (optim/sgd.cpp:34-263, SparseOptimizer::optimize_raw sparse_optimizer.h:42).
 *
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 * Every entry point returns an int status (STG_OK == 0, < 0 on error) and
 * never throws; stg_last_error() returns a thread-local message.  The C++
 * shim in stg/compressor.h turns errors back into std::runtime_error, which
 * is what the reference throws (topk.cpp:34, core.cpp:117,193).
 *
 * Device pointers are HIP device (or host-mapped) pointers on the handle's
 * device; `stream` is a hipStream_t passed as void* (NULL = legacy default
 * stream).  Device entry points are asynchronous and never synchronise the
 * host; host entry points copy in, run, copy out and synchronise.
 */
#ifndef STG_CODEC_H
#define STG_CODEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STG_OK 0
#define STG_ERR_INVALID (-1)     /* bad argument (e.g. capacity < k for topk)   */
#define STG_ERR_UNKNOWN (-2)     /* unknown method string                       */
#define STG_ERR_HIP (-3)         /* HIP runtime error                           */
#define STG_ERR_UNSUPPORTED (-4) /* size outside what this build handles        */
#define STG_ERR_DEVICE (-5)      /* device-side failure flag (see stg_check)    */

typedef struct stg_codec *stg_codec_t;
typedef struct stg_sgd *stg_sgd_t;
typedef struct stg_adam *stg_adam_t;

/* Method strings as in the reference factory (core.cpp:110-118).
 * "topk" reproduces the reference's shipped behaviour (the byte-count memcpy
 * of topk.cpp:31 and idx = 0..k-1); "topk_exact" is the intended top-k by
 * |x| over the whole bucket with real indices.  Replaces the
 * ThresholdvCompressor16 / ThresholdvCompressor / TopkCompressor
 * constructors (thresholdv16.h:33, thresholdv.h:25, topk.h:28). */
int stg_codec_create(const char *method, int device, stg_codec_t *out);
int stg_codec_destroy(stg_codec_t h);
/* Compressor::name() (compressor.h:28): "Thresholdv16", "Thresholdv", "Topk". */
const char *stg_codec_name(stg_codec_t h);

/* Compressor::compress on host memory (compressor.h:30), the engine's MERGE
 * call site (engine/modules/compress.cpp:141) and FasterDpEngine::compress
 * (core.cpp:1210-1245).  Copies src to the device, runs the codec, copies
 * (idx, val) back and synchronises.  *out_count receives compress()'s return
 * value.  `key` is the reference's `name` argument (persistent key
 * "layer@param", task.cpp:56-61); threshold-v ignores it and keys its AIMD
 * state by the src pointer value, as thresholdv.cpp:44 does. */
int stg_codec_compress_host(stg_codec_t h, const char *key, const float *src, size_t n, uint32_t k,
                            uint32_t *dst_idx, size_t idx_cap, float *dst_val, size_t val_cap,
                            int32_t idx_offset, size_t *out_count);

/* Same contract on device-resident buffers, fully asynchronous on `stream`:
 * no host synchronisation, per-key threshold state stays on the device.
 * The returned pair count is written to *d_count (device uint32).  dst
 * buffers are caller-owned with capacity idx_cap (val_cap >= idx_cap). */
int stg_codec_compress_device(stg_codec_t h, const char *key, const float *d_src, size_t n, uint32_t k,
                              uint32_t *d_idx, size_t idx_cap, float *d_val, size_t val_cap,
                              int32_t idx_offset, uint32_t *d_count, void *stream);

/* One bucket of a batched call: the arguments of one compress_device call. */
typedef struct stg_bucket {
    const char *key;
    const float *d_src;
    size_t n;
    uint32_t k;
    uint32_t *d_idx;
    size_t idx_cap;
    float *d_val;
    size_t val_cap;
    int32_t idx_offset;
    uint32_t *d_count;
} stg_bucket_t;

/* Batched compress_device: same results as calling stg_codec_compress_device
 * on buckets[0..nbuckets-1] in order on `stream`.  It stands in for the
 * engine's concurrent MERGE-compress tasks of one iteration (ThreadPool
 * workers calling compress() on different keys, engine/modules/compress.cpp:
 * 141, engine/config.h:7).  thresholdv16 runs up to 32 buckets with distinct
 * keys in one persistent launch, overlapping bucket b's count exchange with
 * bucket b+1's streaming pass; a repeated key starts a new launch. */
int stg_codec_compress_batch_device(stg_codec_t h, const stg_bucket_t *buckets, size_t nbuckets, void *stream);

/* One iteration's MERGE compress tasks with their error feedback
 * (ModuleCompress::run, engine/modules/compress.cpp:139-186): the batched
 * compress above, then for every bucket src[idx[i]] = 0 for i < idx_cap
 * (:178-179; the caller zero-fills idx, compress.cpp:60-64, so unused slots
 * zero element 0 as in the reference) and residual = src (:185), i.e.
 * d_residuals[i] ends as the bucket with the selected entries zeroed and the
 * bucket (d_src, written here) ends identical to it.  thresholdv16 fuses the
 * residual copy into its streaming pass (one HBM read of the bucket instead
 * of two); the other codecs run compress + stg_error_feedback_device. */
int stg_merge_compress_batch_device(stg_codec_t h, const stg_bucket_t *buckets, float *const *d_residuals,
                                    size_t nbuckets, void *stream);

/* One MERGE task with the intra-node gather ahead of it (ModuleCpuGather::run
 * then ModuleCompress::run on local rank r's slice, engine/modules/
 * cpu_gather.cpp:59-87 and compress.cpp:139-186).  bucket->d_src is grad[0]'s
 * slice: it receives d_residual (may be null) + d_grads[1] + ... +
 * d_grads[num_gpus - 1] (slice pointers, [0] ignored, peers' over xGMI) in
 * stg_gather_add_device's order, is compressed, and when d_residual is not
 * null its error feedback runs as in stg_merge_compress_batch_device.  The
 * same results as stg_gather_add_device, then stg_merge_compress_batch_device
 * (d_residual) or stg_codec_compress_device (no residual), on one bucket.
 * thresholdv16 sums the sources inside its one-bucket streaming pass (each
 * source read once, grad[0] stored once, the line sums taken from the sum):
 * one pass instead of the gather's and the codec's.  A key's first call, and
 * the other codecs, run the gather-add pass first.  Async on `stream`. */
int stg_merge_gather_compress_device(stg_codec_t h, const stg_bucket_t *bucket, float *d_residual,
                                     const float *const *d_grads, int num_gpus, void *stream);

/* Batched compress_device whose emission writes the wire form of each stream
 * (comm_manager.cpp:486-590 queueTx's packing, fused into the codec): bucket
 * i's pairs land in d_idx / d_val as stg_wire_encode_device(flags[i]) would
 * write them for the count = min(idx_cap, n) pairs the codec emits -- u16
 * indices when flags[i] & STG_WIRE_U16_IDX, fp16 values when
 * flags[i] & STG_WIRE_F16_VAL (the buffers hold count elements of that type),
 * the codec's own u32 / f32 otherwise.  The same bytes as
 * stg_codec_compress_batch_device followed by one encode per bucket, without
 * the encode pass.  *d_count as in compress_device.  thresholdv16 only
 * (STG_ERR_UNSUPPORTED for the other codecs).  Async on `stream`. */
int stg_codec_compress_wire_batch_device(stg_codec_t h, const stg_bucket_t *buckets, const int *flags,
                                         size_t nbuckets, void *stream);

/* Per-key AIMD state (thresholdv16.cpp:243-259, thresholdv.cpp:72-80), read
 * back for parity tests; synchronises `stream`.  Returns STG_ERR_INVALID when
 * the key has never been compressed.  For threshold-v pass the src pointer
 * value as `key_ptr` (key is ignored); thresholdv16 uses `key`. */
int stg_codec_get_state(stg_codec_t h, const char *key, const void *key_ptr, float *threshold,
                        float *threshold_inc, void *stream);

/* Kernel timing, the GPU analogue of the reference's CRIT_PATH_compress stat
 * span (engine/modules/compress.cpp:140-142, core_module_api.cpp:504-514):
 * when enabled, every codec launch records HIP events on its stream:
 * [0] = the main kernel (thresholdv16: the whole batch kernel; threshold-v and
 * top-k: the streaming/count pass), [1] = the ordering/emission pass (0 for
 * thresholdv16, which has none), [2] = the whole call including first-call
 * work of threshold-v / top-k (thresholdv16's first-call launches precede
 * event [0] and are not timed).  stg_codec_get_timing synchronises the recorded events and returns
 * the accumulated milliseconds [0, 1, 2], the number of launches timed in
 * *calls and resets the accumulators (one batched call = one launch per run of
 * distinct keys). */
int stg_codec_set_timing(stg_codec_t h, int enable);
int stg_codec_get_timing(stg_codec_t h, double *ms3, uint64_t *calls);

/* Diagnostics: the first n (<= 64) scratch words of the handle's workspace
 * for `stream` (phase stamps of builds with STG_FILL_STAMPS); syncs. */
int stg_codec_debug_words(stg_codec_t h, void *stream, uint32_t *out, int n);

/* Checks the device-side failure word of every workspace of this handle
 * (e.g. a regime-B candidate set larger than the build supports); syncs. */
int stg_codec_check(stg_codec_t h);

/* MERGE decompress (cpu_optimize.cpp:40-72): `world` rank streams of
 * `per_rank` (idx, val) pairs each, laid out back to back, are scattered
 * into a dense zeroed scratch of n floats in rank order (index_put_, no
 * accumulate, per rank: of a rank's duplicated indices -- e.g. the wire
 * format's u16 saturation -- the last occurrence wins), summed, divided by
 * `world`, and gathered at the union of indices (one entry per index,
 * unique1d :14-24).  world > 1: output index-ascending, d_dense (n floats,
 * zero) and d_mark (n bytes, zero, 16-byte aligned) are caller scratch and
 * are left zero.  world == 1: no dense scratch; the winners in stream order.
 * Indices >= n are dropped.  *d_out_count (device) gets the union size
 * (0xffffffff after a device failure).  Internal scratch is kept per (device,
 * stream) for reuse: 4 B per element of the largest n seen (8 B when world >
 * 1) plus 12 B per 4,096-pair tile -- about 64 MiB for n = 16 Mi at world 1,
 * 128 MiB at world > 1 -- until stg_scatter_merge_release. */
int stg_scatter_merge_device(const uint32_t *d_idx, const float *d_val, size_t per_rank, int world, size_t n,
                             float *d_dense, uint8_t *d_mark, uint32_t *d_out_idx, float *d_out_val,
                             uint32_t *d_out_count, void *stream);
/* The MERGE decompress scratch of (current device, stream): syncs the stream
 * and returns STG_ERR_DEVICE if a call on it hit a device failure (sticky). */
int stg_scatter_merge_check(void *stream);
/* Frees the MERGE decompress scratch of (current device, stream) after its
 * work is done (call it before destroying a stream that merged). */
int stg_scatter_merge_release(void *stream);

/* Error feedback of the MERGE compress (engine/modules/compress.cpp:172-186):
 * after compressing d_grad into numel (idx, val) slots, zero d_grad at every
 * d_idx[i], i < numel (unwritten slots hold index 0, so element 0 is zeroed
 * too, as in the reference), and copy the bucket into d_residual.  Both
 * arrays end identical.  Asynchronous on `stream`. */
int stg_error_feedback_device(float *d_grad, size_t n, const uint32_t *d_idx, size_t numel, float *d_residual,
                              void *stream);

/* Sparse SGD (optim/sgd.cpp:34-263 scalar path; options sgd.cpp:265-300).
 * optimize_raw() keeps one momentum buffer per `name` on the device. */
int stg_sgd_create(int device, float lr, float momentum, float dampening, float weight_decay, int nesterov,
                   int maximize, stg_sgd_t *out);
int stg_sgd_destroy(stg_sgd_t o);
int stg_sgd_optimize_raw_device(stg_sgd_t o, const char *name, float *d_param, uint32_t param_len,
                                const float *d_grad, const uint32_t *d_idx, uint32_t grad_len,
                                const uint32_t *d_grad_len, void *stream);
int stg_sgd_get_momentum(stg_sgd_t o, const char *name, float *host_out, uint32_t len, void *stream);
/* ModuleCpuOptimize::run (engine/modules/cpu_optimize.cpp:26-100): the MERGE
 * decompress of the received stream (as stg_scatter_merge_device: d_out_idx /
 * d_out_val / d_out_count get the merged stream, param_len is n) followed by
 * SparseOptimizer::optimize_raw of `o` on it (sgd.cpp:34-263), in one call.
 * world == 1: two launches, the election and the emission with every winner's
 * step in the same pass (each index is elected once, so the updates commute;
 * parameters and momentum bitwise equal to the two separate calls); world > 1:
 * the two calls, the step's length read from d_out_count on the device. */
int stg_merge_optimize_sgd_device(stg_sgd_t o, const char *name, float *d_param, uint32_t param_len,
                                  const uint32_t *d_idx, const float *d_val, size_t per_rank, int world,
                                  float *d_dense, uint8_t *d_mark, uint32_t *d_out_idx, float *d_out_val,
                                  uint32_t *d_out_count, void *stream);
/* The same with Adam (adam.cpp:19-86): world 1 without amsgrad runs the step
 * inside the emission launch; amsgrad (its running maximum is an ordered scan)
 * and world > 1 run the decompress, then stg_adam_optimize_raw_device. */
int stg_merge_optimize_adam_device(stg_adam_t o, const char *name, float *d_param, uint32_t param_len,
                                   const uint32_t *d_idx, const float *d_val, size_t per_rank, int world,
                                   float *d_dense, uint8_t *d_mark, uint32_t *d_out_idx, float *d_out_val,
                                   uint32_t *d_out_count, void *stream);

/* Sparse Adam (optim/adam.cpp:19-86; options Adam::configure adam.cpp:90-122,
 * defaults adam.h:21-23, lr sparse_optimizer.h:30).  optimize_raw() keeps per
 * `name` the m and v arrays (param_len floats, zeroed), the amsgrad running
 * max vmax (a float, 0) on the device and the tick (1, +1 per call) on the
 * host, as adam.cpp:28-35,81-82.  Indices must be unique within a call (every
 * codec output and the MERGE union are); with amsgrad grad_len <= param_len.
 * Calls on one name are serialised by the caller's stream (the reference holds
 * a mutex, adam.cpp:47).  get_state copies m, v (len floats each) and vmax to
 * the host after synchronising `stream`, and returns the next call's tick
 * through *tick_out; STG_ERR_INVALID before the name's first call. */
int stg_adam_create(int device, float lr, float b1, float b2, float eps, float weight_decay, int amsgrad,
                    int maximize, stg_adam_t *out);
int stg_adam_destroy(stg_adam_t o);
int stg_adam_optimize_raw_device(stg_adam_t o, const char *name, float *d_param, uint32_t param_len,
                                 const float *d_grad, const uint32_t *d_idx, uint32_t grad_len,
                                 const uint32_t *d_grad_len, void *stream);
int stg_adam_get_state(stg_adam_t o, const char *name, float *host_m, float *host_v, uint32_t len,
                       float *host_vmax, uint32_t *tick_out, void *stream);
/* Synchronises `stream` and reports the handle's sticky device failure word:
 * STG_ERR_DEVICE if an amsgrad look-back ever timed out (its updates used an
 * incomplete running max), STG_OK otherwise. */
int stg_adam_check(stg_adam_t o, void *stream);

/* Intra-node gather-add before the codec (ModuleCpuGather::run,
 * engine/modules/cpu_gather.cpp:59-87, add_arrays misc/array_util.h:12-54).
 * stg_gather_slice gives local rank r's slice [n*r/N, n*(r+1)/N).  add: over
 * that slice, d_grad0 += d_residual, then += d_grads[1], ..., d_grads[N-1]
 * (d_grads is a host array of N device pointers; [0] is ignored, it is
 * d_grad0), in that order per element, in one pass.  Sources may be peer
 * GPUs' buffers when P2P access is enabled (xGMI).  d_residual may be null
 * (no residual term; differs from adding zeros only for -0.0 elements).
 * N <= 16.  Async on `stream`. */
int stg_gather_slice(uint64_t n, int local_rank, int num_gpus, uint64_t *start, uint64_t *end);
int stg_gather_add_device(float *d_grad0, const float *d_residual, const float *const *d_grads, int num_gpus,
                          uint64_t n, int local_rank, void *stream);

/* Wire format of the compressed stream (engine/comm_manager.cpp:486-590).
 * stg_wire_flag returns the flag byte queueTx would send (comm_manager.cpp:
 * 573-590, comm_manager.h:24-25): STG_WIRE_U16_IDX when tensor_numel < 65536,
 * STG_WIRE_F16_VAL when fp16_values (FP16_COMPRESSION, config.h:64).
 * encode writes numel indices as uint16 (flag & 1) or uint32 and numel values
 * as fp16 bits (flag & 2) or float; decode is the receiver's inverse
 * (comm_manager.cpp:877-906).  Both reproduce the reference's bytes exactly,
 * including its SIMD-block / scalar-tail differences (wire.hip).  Async. */
#define STG_WIRE_U16_IDX 0x01
#define STG_WIRE_F16_VAL 0x02
int stg_wire_flag(uint64_t tensor_numel, int fp16_values);
int stg_wire_encode_device(const uint32_t *d_idx, const float *d_val, size_t numel, int flag, void *d_idx_out,
                           void *d_val_out, void *stream);
int stg_wire_decode_device(const void *d_idx_in, const void *d_val_in, size_t numel, int flag, uint32_t *d_idx,
                           float *d_val, void *stream);

/* One wire stream of a batched encode: the arguments of one encode call. */
typedef struct stg_wire_stream {
    const uint32_t *d_idx;
    const float *d_val;
    size_t numel;
    int flag;
    void *d_idx_out;
    void *d_val_out;
} stg_wire_stream_t;

/* Batched stg_wire_encode_device: the same bytes as encoding streams[0..n-1]
 * one by one (the tx queue of one iteration, comm_manager.cpp:573-640), in
 * launches of up to 16 streams instead of one launch per stream. */
int stg_wire_encode_batch_device(const stg_wire_stream_t *streams, size_t nstreams, void *stream);

/* Synthetic fp32 buckets from the integer-only generator of SURVEY 8(d)
 * (dist 0 = D1, 1 = D2 heavy tail, 2 = D3 zeros with prob param/1e4);
 * bit-identical to oracle/stg_oracle.cpp:orc_synth_fill. */
int stg_synth_fill_device(float *d_dst, size_t n, uint64_t seed, int dist, uint32_t param, void *stream);

/* Thread-local message for the last failing call on this thread. */
const char *stg_last_error(void);

#ifdef __cplusplus
}
#endif

#endif /* STG_CODEC_H */
