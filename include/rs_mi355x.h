/*
 * rs_mi355x.h -- C ABI of the MI355X (gfx950) Reed-Solomon GF(2^16) engine.
 *
 * Drop-in boundary for AndersTrier/reed-solomon-simd v3.1.0 (reference mounted
 * at /root/reference; paths below are relative to it).  Plain pointers and
 * sizes only; device pointers are HIP device allocations, `stream` is a
 * hipStream_t passed as void* (NULL = default stream).
 *
 *   reference item                                   replaced by
 *   -----------------------------------------------  ------------------------------
 *   Error enum + fields        src/lib.rs:48-142     rs_status / rs_error
 *   encode()/decode()          src/lib.rs:251-353    rs_encode / rs_decode (host buffers)
 *   ReedSolomonEncoder         src/reed_solomon.rs:13-81
 *     ::new / ::reset / ::supports                    rs_encoder_new / _reset / rs_supports
 *     ::add_original_shard                            rs_encoder_add_original_shard
 *     ::encode -> EncoderResult                       rs_encoder_encode
 *     EncoderResult::recovery  src/encoder_result.rs:17-33   rs_encoder_recovery
 *     EncoderResult Drop (reset_received)             rs_encoder_result_drop
 *   ReedSolomonDecoder         src/reed_solomon.rs:83-183
 *     ::add_original_shard / ::add_recovery_shard     rs_decoder_add_*_shard
 *     ::decode -> DecoderResult                       rs_decoder_decode
 *     DecoderResult::restored_original src/decoder_result.rs:17-33  rs_decoder_restored_original
 *   DefaultRate / HighRate / LowRate  src/rate/rate_*.rs  rs_rate (RS_RATE_DEFAULT/HIGH/LOW)
 *   trait Engine               src/engine.rs:234-291
 *     fft / ifft (ShardsRefMut, pos, size, trunc, skew_delta)  rs_engine_fft / rs_engine_ifft
 *     mul(x, log_m)                                   rs_engine_mul
 *     eval_poly(erasures, truncated)                  rs_engine_eval_poly (host array)
 *   tables::get_exp_log / get_skew  src/engine/tables.rs:98-165  rs_table_exp/log/skew
 *
 * Device-resident batch entry points (the performance path; no reference
 * counterpart because the reference engine only sees host slices):
 *   rs_encode_device / rs_decode_device (+ _strided, + _batch: many
 *   stripes of one shape in one launch)
 *
 * Thread-safety: a context may be shared by threads (like DefaultEngine:
 * Send + Sync, src/lib.rs:385-409): calls on one context are serialized on the
 * host by an internal mutex, and the device scratch is kept per (context,
 * stream), so calls enqueued on different streams may execute concurrently on
 * the device.  Do not destroy a stream while calls on it are in flight and
 * then pass a new stream that reuses its handle.  A context keeps the scratch
 * of at most RS_MAX_STREAM_WORKSPACES streams (device buffers sized to the
 * largest call made on each, plus pinned staging); a call on a further stream
 * takes over the least recently used stream's scratch (buffers kept, no free)
 * after waiting for that stream's last call -- by an event recorded at the end
 * of each call once 8 or more streams are in use, else by synchronizing the
 * device.  rs_release_stream_scratch frees one stream's scratch at once (call
 * it before destroying a stream the context has seen).  Single-level HighRate
 * encodes with several chunks and few packs spread the chunks over the grid,
 * with a work buffer of about the input's size, only up to 256 MiB of it; larger
 * ones run the chunks in sequence without one.  Every entry point runs on
 * the context's device and restores the calling thread's current device.  An
 * encoder/decoder handle is used by one thread at a time (like
 * &mut ReedSolomonEncoder).
 */
#ifndef RS_MI355X_H
#define RS_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Error codes, one per reference Error variant (src/lib.rs:48-142). */
typedef enum rs_status {
    RS_OK = 0,
    RS_ERR_DIFFERENT_SHARD_SIZE = 1,            /* shard_bytes, got */
    RS_ERR_DUPLICATE_ORIGINAL_SHARD_INDEX = 2,  /* index */
    RS_ERR_DUPLICATE_RECOVERY_SHARD_INDEX = 3,  /* index */
    RS_ERR_INVALID_ORIGINAL_SHARD_INDEX = 4,    /* original_count, index */
    RS_ERR_INVALID_RECOVERY_SHARD_INDEX = 5,    /* recovery_count, index */
    RS_ERR_INVALID_SHARD_SIZE = 6,              /* shard_bytes */
    RS_ERR_NOT_ENOUGH_SHARDS = 7,               /* original_count, original_received_count, recovery_received_count */
    RS_ERR_TOO_FEW_ORIGINAL_SHARDS = 8,         /* original_count, original_received_count */
    RS_ERR_TOO_MANY_ORIGINAL_SHARDS = 9,        /* original_count */
    RS_ERR_UNSUPPORTED_SHARD_COUNT = 10,        /* original_count, recovery_count */
    /* not in the reference: */
    RS_ERR_DEVICE = 100,                        /* HIP runtime failure (message via rs_last_device_error) */
    RS_ERR_INVALID_ARGUMENT = 101               /* null handle / pointer, or unsupported device-API layout */
} rs_status;

/* Error payload; fields not used by a variant are 0.  Field names follow the
 * reference variants' fields. */
typedef struct rs_error {
    int32_t code; /* rs_status */
    uint64_t original_count;
    uint64_t recovery_count;
    uint64_t shard_bytes;
    uint64_t got;
    uint64_t index;
    uint64_t original_received_count;
    uint64_t recovery_received_count;
} rs_error;

typedef enum rs_rate { RS_RATE_DEFAULT = 0, RS_RATE_HIGH = 1, RS_RATE_LOW = 2 } rs_rate;

typedef struct rs_context rs_context;
typedef struct rs_encoder rs_encoder;
typedef struct rs_decoder rs_decoder;
typedef struct rs_encoder_work rs_encoder_work; /* EncoderWork (src/rate/encoder_work.rs) */
typedef struct rs_decoder_work rs_decoder_work; /* DecoderWork (src/rate/decoder_work.rs) */

/* ---- context: one per device; builds and uploads the GF tables once ---- */
rs_status rs_context_create(int device, rs_context **out);
void rs_context_destroy(rs_context *ctx);
const char *rs_last_device_error(void);
const char *rs_version(void);

/* ---- capability / validation (src/rate/rate_default.rs:15-64, src/rate.rs:91-106) ---- */
int rs_supports(rs_rate rate, uint64_t original_count, uint64_t recovery_count);
/* 1 = HighRate, 0 = LowRate, -1 = unsupported */
int rs_use_high_rate(uint64_t original_count, uint64_t recovery_count);
rs_status rs_validate(rs_rate rate, uint64_t original_count, uint64_t recovery_count, uint64_t shard_bytes,
                      rs_error *err);
/* work_count of the encoder / decoder (rate_high.rs:135-141, 308-312; rate_low.rs same) */
uint64_t rs_encoder_work_count(rs_rate rate, uint64_t original_count, uint64_t recovery_count);
uint64_t rs_decoder_work_count(rs_rate rate, uint64_t original_count, uint64_t recovery_count);

/* ---- one-shot host API (src/lib.rs:251-353) ----
 * rs_encode: `original` = array of original_count pointers to shard_bytes each;
 *   recovery_out = recovery_count * shard_bytes contiguous.
 * rs_decode: original/recovery = arrays of (index, pointer) given as parallel
 *   arrays; restored_out = original_count * shard_bytes, only missing rows
 *   written; restored_mask (original_count bytes) set to 1 for restored rows. */
rs_status rs_encode(rs_context *ctx, uint64_t original_count, uint64_t recovery_count, uint64_t shard_bytes,
                    const uint8_t *const *original, uint64_t original_given, uint8_t *recovery_out, rs_error *err);
rs_status rs_decode(rs_context *ctx, uint64_t original_count, uint64_t recovery_count, uint64_t shard_bytes,
                    const uint64_t *original_index, const uint8_t *const *original, uint64_t original_given,
                    const uint64_t *recovery_index, const uint8_t *const *recovery, uint64_t recovery_given,
                    uint8_t *restored_out, uint8_t *restored_mask, rs_error *err);

/* ---- ReedSolomonEncoder / RateEncoder (src/reed_solomon.rs, src/rate.rs:113-173) ---- */
rs_status rs_encoder_new(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                         uint64_t shard_bytes, rs_encoder **out, rs_error *err);
rs_status rs_encoder_reset(rs_encoder *enc, uint64_t original_count, uint64_t recovery_count,
                           uint64_t shard_bytes, rs_error *err);
rs_status rs_encoder_add_original_shard(rs_encoder *enc, const uint8_t *shard, uint64_t len, rs_error *err);
rs_status rs_encoder_encode(rs_encoder *enc, rs_error *err);
/* valid after a successful encode until rs_encoder_result_drop / next mutation;
 * NULL when index >= recovery_count (src/rate/encoder_work.rs:90-96) */
const uint8_t *rs_encoder_recovery(rs_encoder *enc, uint64_t index);
void rs_encoder_result_drop(rs_encoder *enc); /* EncoderResult::drop -> reset_received */
int rs_encoder_is_high_rate(const rs_encoder *enc);
void rs_encoder_free(rs_encoder *enc);
/* RateEncoder::into_parts (src/rate.rs:129-131): consumes enc (freed), returns its engine
 * (the context) and its working space (host and device buffers) for reuse by another
 * encoder of any rate and shape.  Either out pointer may be NULL.  The work remembers
 * the device of the context it came from: handed to a context on another device, its
 * device buffers are freed (not reused) and only its host buffers are kept. */
rs_status rs_encoder_into_parts(rs_encoder *enc, rs_context **ctx_out, rs_encoder_work **work_out);
/* RateEncoder::new with `work: Option<EncoderWork>` (src/rate.rs:133-139,
 * src/rate/rate_high.rs:93-103): like
 * rs_encoder_new, reusing `work`'s buffers (NULL = none).  `work` is consumed in every
 * case, also when the call fails (as when the reference's new returns Err). */
rs_status rs_encoder_new_with_work(rs_context *ctx, rs_rate rate, uint64_t original_count,
                                   uint64_t recovery_count, uint64_t shard_bytes, rs_encoder_work *work,
                                   rs_encoder **out, rs_error *err);
void rs_encoder_work_free(rs_encoder_work *work);

/* ---- ReedSolomonDecoder / RateDecoder (src/reed_solomon.rs, src/rate.rs:179-250) ---- */
rs_status rs_decoder_new(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                         uint64_t shard_bytes, rs_decoder **out, rs_error *err);
rs_status rs_decoder_reset(rs_decoder *dec, uint64_t original_count, uint64_t recovery_count,
                           uint64_t shard_bytes, rs_error *err);
rs_status rs_decoder_add_original_shard(rs_decoder *dec, uint64_t index, const uint8_t *shard, uint64_t len,
                                        rs_error *err);
rs_status rs_decoder_add_recovery_shard(rs_decoder *dec, uint64_t index, const uint8_t *shard, uint64_t len,
                                        rs_error *err);
rs_status rs_decoder_decode(rs_decoder *dec, rs_error *err);
/* NULL unless original `index` was missing and has been restored
 * (src/rate/decoder_work.rs:189-197) */
const uint8_t *rs_decoder_restored_original(rs_decoder *dec, uint64_t index);
uint64_t rs_decoder_restored_count(const rs_decoder *dec);
void rs_decoder_result_drop(rs_decoder *dec); /* DecoderResult::drop -> reset_received */
int rs_decoder_is_high_rate(const rs_decoder *dec);
void rs_decoder_free(rs_decoder *dec);
/* RateDecoder::into_parts / new with work (src/rate.rs:206-218, src/rate/rate_high.rs:260-270):
 * as for the encoder. */
rs_status rs_decoder_into_parts(rs_decoder *dec, rs_context **ctx_out, rs_decoder_work **work_out);
rs_status rs_decoder_new_with_work(rs_context *ctx, rs_rate rate, uint64_t original_count,
                                   uint64_t recovery_count, uint64_t shard_bytes, rs_decoder_work *work,
                                   rs_decoder **out, rs_error *err);
void rs_decoder_work_free(rs_decoder_work *work);

/* ---- device-resident batch path (HBM in, HBM out) ----
 * d_original: original_count rows, d_recovery: recovery_count rows, both
 * row-major with row stride shard_bytes.  shard_bytes: any positive even
 * size (Error::InvalidShardSize otherwise); whole 64-byte blocks use the
 * reference's block layout (algorithm.md:18-31) and the last S % 64 bytes its
 * tail layout (S % 64 / 2 low bytes, then the high bytes: src/engine/shards.rs:38-74),
 * so shards are byte-identical to the reference's Encoder / Decoder output.
 * Asynchronous on `stream` (device scratch per context and stream: see
 * "Thread-safety" above). */
rs_status rs_encode_device(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                           uint64_t shard_bytes, const void *d_original, void *d_recovery, void *stream,
                           rs_error *err);
/* original_present / recovery_present: HOST arrays of 0/1 bytes.
 * d_restored: original_count rows; only missing originals are written.
 * Missing rows of d_original / d_recovery are never read. */
rs_status rs_decode_device(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                           uint64_t shard_bytes, const void *d_original, const uint8_t *original_present,
                           const void *d_recovery, const uint8_t *recovery_present, void *d_restored, void *stream,
                           rs_error *err);
/* Column slices of wider matrices: shard r of a matrix starts at base + r * stride
 * (stride 0 = shard_bytes; otherwise >= shard_bytes).  Any alignment works:
 * when a base address or stride is not a multiple of 4 the kernels access the
 * caller's matrices byte by byte (slower).  Every engine op is column-wise
 * (src/engine/utils.rs:35-43), so encoding a range of whole 64-byte blocks of
 * each shard yields exactly those blocks of the full recovery shards: the
 * building block of the column-partitioned multi-GPU encode. */
rs_status rs_encode_device_strided(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                                   uint64_t shard_bytes, const void *d_original, uint64_t original_stride,
                                   void *d_recovery, uint64_t recovery_stride, void *stream, rs_error *err);
rs_status rs_decode_device_strided(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                                   uint64_t shard_bytes, const void *d_original, uint64_t original_stride,
                                   const uint8_t *original_present, const void *d_recovery, uint64_t recovery_stride,
                                   const uint8_t *recovery_present, void *d_restored, uint64_t restored_stride,
                                   void *stream, rs_error *err);
/* A batch of `stripes` independent stripes of one shape (MI355X extension: a
 * storage node codes many stripes at once).  Stripe b's original matrix starts
 * at d_original + b * original_stripe_stride bytes (0 = original_count rows of
 * the row stride), likewise for the recovery / restored matrices; row strides
 * as in the _strided calls.  Where one stripe runs as a single column-kernel
 * launch the whole batch is one launch (stripes x shard_bytes / 8 workgroups);
 * otherwise the stripes run one after another.  Result: identical to
 * `stripes` separate calls.  The decode applies ONE erasure pattern to every
 * stripe (a failed device loses the same shard indices in all of them). */
rs_status rs_encode_device_batch(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                                 uint64_t shard_bytes, uint64_t stripes, const void *d_original,
                                 uint64_t original_stride, uint64_t original_stripe_stride, void *d_recovery,
                                 uint64_t recovery_stride, uint64_t recovery_stripe_stride, void *stream,
                                 rs_error *err);
rs_status rs_decode_device_batch(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                                 uint64_t shard_bytes, uint64_t stripes, const void *d_original,
                                 uint64_t original_stride, uint64_t original_stripe_stride,
                                 const uint8_t *original_present, const void *d_recovery, uint64_t recovery_stride,
                                 uint64_t recovery_stripe_stride, const uint8_t *recovery_present, void *d_restored,
                                 uint64_t restored_stride, uint64_t restored_stripe_stride, void *stream,
                                 rs_error *err);

/* ---- host-memory pipeline (shards arrive from a socket or file) ----
 * h_original (original_count x shard_bytes) and h_recovery (recovery_count x
 * shard_bytes) are row-major HOST matrices; pinned memory (rs_host_alloc,
 * hipHostMalloc) gives full PCIe rate, pageable memory works but is staged by
 * the runtime.  The byte axis is cut into `slices` column slices of whole
 * 64-byte blocks (0 = 1); slice k is copied in, coded and copied out on its
 * own stream, overlapping neighbouring slices.  Blocking: returns when the
 * outputs are in host memory.  shard_bytes: any even size (the tail block
 * travels with the last slice).
 * Decode copies in only received rows and writes only the missing originals
 * of h_restored (original_count x shard_bytes). */
void *rs_host_alloc(uint64_t bytes);
void rs_host_free(void *p);
rs_status rs_encode_host(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                         uint64_t shard_bytes, const void *h_original, void *h_recovery, uint32_t slices,
                         rs_error *err);
rs_status rs_decode_host(rs_context *ctx, rs_rate rate, uint64_t original_count, uint64_t recovery_count,
                         uint64_t shard_bytes, const void *h_original, const uint8_t *original_present,
                         const void *h_recovery, const uint8_t *recovery_present, void *h_restored,
                         uint32_t slices, rs_error *err);

/* ---- Engine trait over a device shard matrix (src/engine.rs:234-291) ----
 * d_rows: shard_count rows of shard_len_64 64-byte blocks (ShardsRefMut,
 * src/engine/shards.rs:100-189).  Infallible in the reference (debug_assert on
 * bad args); here bad args return RS_ERR_INVALID_ARGUMENT.  Semantics are
 * engine_naive.rs:43-105 for every row, including rows at and past
 * truncated_size (only the butterfly groups that start below it are
 * transformed). */
rs_status rs_engine_fft(rs_context *ctx, void *d_rows, uint64_t shard_count, uint64_t shard_len_64, uint64_t pos,
                        uint64_t size, uint64_t truncated_size, uint64_t skew_delta, void *stream);
rs_status rs_engine_ifft(rs_context *ctx, void *d_rows, uint64_t shard_count, uint64_t shard_len_64, uint64_t pos,
                         uint64_t size, uint64_t truncated_size, uint64_t skew_delta, void *stream);
rs_status rs_engine_mul(rs_context *ctx, void *d_rows, uint64_t block_count, uint16_t log_m, void *stream);
/* host array of 65536 elements, in place (src/engine/utils.rs:20-31) */
void rs_engine_eval_poly(uint16_t *erasures, uint64_t truncated_size);
/* formal derivative over all shard_count rows (src/engine/utils.rs:99-104) */
rs_status rs_engine_formal_derivative(rs_context *ctx, void *d_rows, uint64_t shard_count, uint64_t shard_len_64,
                                      void *stream);

/* ---- Engine trait over a HOST shard array: the reference's own calling convention ----
 * `rows` is the host storage of a ShardsRefMut (shard_count x shard_len_64 64-byte
 * blocks, src/engine/shards.rs:100-189); Engine::fft / ifft (src/engine.rs:119-151)
 * transform rows [pos, pos + size) and Engine::mul (src/engine.rs:154) scales
 * block_count blocks.  Blocking: the rows are copied to the device, transformed
 * with the same kernels as rs_engine_fft / rs_engine_ifft / rs_engine_mul, and
 * copied back.  This is what a Rust `impl Engine` binds; it pays a
 * PCIe round trip per call, the device-resident calls above do not. */
rs_status rs_engine_fft_host(rs_context *ctx, uint8_t *rows, uint64_t shard_count, uint64_t shard_len_64,
                             uint64_t pos, uint64_t size, uint64_t truncated_size, uint64_t skew_delta);
rs_status rs_engine_ifft_host(rs_context *ctx, uint8_t *rows, uint64_t shard_count, uint64_t shard_len_64,
                              uint64_t pos, uint64_t size, uint64_t truncated_size, uint64_t skew_delta);
rs_status rs_engine_mul_host(rs_context *ctx, uint8_t *blocks, uint64_t block_count, uint16_t log_m);

/* Device scratch of one stream (see "Thread-safety"): synchronizes `stream`
 * and frees the context's scratch for it.  The stream must still be valid. */
#define RS_MAX_STREAM_WORKSPACES 16
rs_status rs_release_stream_scratch(rs_context *ctx, void *stream);

/* ---- kernel timing (bench instrumentation, not a reference item) ----
 * While enabled, every kernel the context launches is bracketed by HIP events
 * on the stream it is launched on.  rs_profile_collect synchronizes those
 * events and returns, in launch order, each launch's duration (ms), its
 * kernel name and the algorithmic HBM bytes of that launch (rows it must read
 * from memory + rows it writes, times the row size); then clears the record.
 * Returns the number of records written (<= max). */
rs_status rs_profile_enable(rs_context *ctx, int enable);
int rs_profile_collect(rs_context *ctx, float *ms, uint64_t *bytes, const char **names, int max);

/* ---- device check ----
 * rs_check_device synchronizes the context's device and returns
 * RS_ERR_DEVICE (message in rs_last_device_error) if an earlier asynchronous
 * launch failed, else RS_OK. */
rs_status rs_check_device(rs_context *ctx);

/* ---- column kernel control (engine tuning, not a reference item) ----
 * Transforms of 2^7 .. 2^12 rows over at most RS_MI355X_MONO_MAX_PACKS (256)
 * packs of 4 elements run as one launch in which a workgroup owns every row
 * of one pack (DESIGN.md "Column kernel").  rs_mono_enable(ctx, 0) selects
 * the pass kernels instead (also: RS_MI355X_NO_MONO=1 at context
 * creation); 1 (default) uses it where it is fastest (single-chunk transforms
 * of 2^7 .. 2^10 rows, twiddles staged in LDS); 2 also for multi-chunk and
 * 2^11 / 2^12-row transforms (also: RS_MI355X_MONO_ALL=1).  Adding 4 turns off
 * the split decode plan of 2^9 .. 2^11-row decodes whose restored rows lie in
 * one half of the work rows (also: RS_MI355X_NO_SPLIT=1).  Single-chunk
 * encodes and decodes of at most half the device's CU count of 4-element packs
 * use packs of 2 elements (twice the workgroups; RS_MI355X_E2_MAX_PACKS sets
 * the limit): adding 8 keeps 4-element packs, adding 16 uses 2-element packs
 * for every single-chunk launch.  Single-chunk 2-element encodes of 2^8 and 2^9
 * rows run on the one-row-per-lane kernel (rs_lane.hip; RS_MI355X_LANE=0 at
 * context creation: never); adding 32 also runs 2^10-row ones there, adding 64
 * none.  Adding 128 runs single-chunk transforms of 2^12 rows as two launches
 * of the 2^11-row kernel split by halves of the rows (off by default: slower
 * than the pass kernels; RS_MI355X_HALF=1 at context creation: on), adding 256
 * turns that off again.  Multi-chunk encodes of 2^2 .. 2^7-row transforms
 * (HighRate N > pow2(M), LowRate M > pow2(N)) run as one launch whose waves
 * take the chunks in parallel (rs_chunks.hip; RS_MI355X_CHUNKS=0 at context
 * creation: never) where that measured faster: all of them but LowRate
 * encodes of more than 8 output chunks in 2-element packs.  Adding 512 sends
 * every multi-chunk encode of those sizes there, adding 1024 none.  Adding
 * 2048 runs single-chunk 2-element encodes of 2^10 rows as the 4-element
 * kernel of 2^9 pair rows (the quad encode; off by default: bit-exact but
 * slower; RS_MI355X_QUAD=1 at context creation: on), adding 4096 turns it off.
 * Neither bit of a pair: the context's defaults (its environment included).
 * A/B and tests; results are identical in every mode. */
rs_status rs_mono_enable(rs_context *ctx, int enable);

/* ---- GF(2^16) tables (src/engine/tables.rs), host copies ---- */
const uint16_t *rs_table_exp(void);       /* 65536 */
const uint16_t *rs_table_log(void);       /* 65536 */
const uint16_t *rs_table_skew(void);      /* 65535 */
const uint16_t *rs_table_log_walsh(void); /* 65536 */
/* this engine's byte-permute multiply tables, 20 words per entry, 65536
 * entries (format: reed-solomon-simd_amd/csrc/gf_tables.cpp fill_perm) */
const uint32_t *rs_table_perm_by_log(void);
const uint32_t *rs_table_perm_by_skew(void);

#ifdef __cplusplus
}
#endif
#endif
