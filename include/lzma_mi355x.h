/*
 * lzma_mi355x.h -- C ABI of the MI355X-native LZMA encode/decode path.
 *
 * This is the drop-in boundary for the hot path of rfalke/lzma-java
 * (src/main/java/SevenZip/Compression/LZMA/Encoder.java and Decoder.java).
 * Plain C types only: no torch, no HIP types in the signatures (streams are
 * passed as void*). A JNI shim binds these entry points
 * for the Java drop-in classes SevenZip.Compression.LZMA.Encoder/Decoder.
 *
 * Reference interface each entry point replaces:
 *   lzma_params_default   Encoder() field defaults          Encoder.java:135-160
 *   lzma_params_check     Encoder setters' range checks      Encoder.java:1135-1180
 *   lzma_write_props      Encoder.WriteCoderProperties       Encoder.java:1079-1085
 *   lzma_read_props       Decoder.SetDecoderProperties       Decoder.java:303-318
 *   lzma_encode           Encoder.Code (one stream)          Encoder.java:1064-1077
 *   lzma_enc_batch[_dev]  Encoder.Code on N independent streams
 *   lzma_pack_dev         (framing) contiguous multi-stream container
 *   lzma_decode           Decoder.Code (one stream)          Decoder.java:205-301
 *   lzma_dec_batch[_dev]  Decoder.Code on N independent streams
 *   lzma_*_batch_multi    the batch entry points over a device mask
 *   lzma_match_lists      BinTree.GetMatches at every position (diagnostic)  BinTree.java:152-273
 *   lzma_bench_generate   LzmaBench.CBenchRandomGenerator    LzmaBench.java:15-127
 *
 * Every encoded stream is byte-identical to Encoder.Code on the same bytes
 * with the same parameters: raw range-coder bytes, no 13-byte .lzma header
 * (the header is written by the caller, LzmaAlone.java:208-217).
 * Errors are returned as status codes; nothing throws across the ABI.
 */
#ifndef LZMA_MI355X_H
#define LZMA_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LZMA_OK 0
#define LZMA_E_PARAM (-1)     /* a setter would have returned false */
#define LZMA_E_NOMEM (-2)     /* host or device allocation failed */
#define LZMA_E_DEVICE (-3)    /* HIP runtime error */
#define LZMA_E_OVERFLOW (-4)  /* output capacity too small */
#define LZMA_E_DATA (-5)      /* corrupt stream: Decoder.Code returned false */
#define LZMA_E_NODEVICE (-6)  /* no HIP device: the product path has no CPU fallback */
#define LZMA_E_INTERNAL (-7)

typedef struct lzma_params {
    int32_t dict_size; /* 1 .. 2^29            (Encoder.SetDictionarySize) */
    int32_t fb;        /* 5 .. 273             (Encoder.SetNumFastBytes) */
    int32_t mf;        /* 0=bt2 1=bt4 2=bt4b   (Encoder.SetMatchFinder) */
    int32_t lc;        /* 0 .. 8               (Encoder.SetLcLpPb) */
    int32_t lp;        /* 0 .. 4 */
    int32_t pb;        /* 0 .. 4 */
    int32_t eos;       /* end marker           (Encoder.SetEndMarkerMode) */
} lzma_params;

typedef struct lzma_ctx lzma_ctx;

const char *lzma_version(void);
int lzma_params_default(lzma_params *p);
int lzma_params_check(const lzma_params *p);
int lzma_write_props(const lzma_params *p, uint8_t out[5]);
int lzma_read_props(const uint8_t in[5], lzma_params *p);
/* Output capacity that always suffices for one encoded stream of n bytes. */
uint64_t lzma_enc_bound(uint64_t n);

int lzma_ctx_create(int device, lzma_ctx **out);
void lzma_ctx_destroy(lzma_ctx *ctx);
const char *lzma_last_error(const lzma_ctx *ctx);
/* Upper bound on input bytes processed per device pass (workspace sizing). */
int lzma_ctx_set_batch_bytes(lzma_ctx *ctx, uint64_t bytes);
/* Per-kernel timing with HIP events on the launch stream (0 = off). */
int lzma_ctx_set_timing(lzma_ctx *ctx, int on);
/* names[i] / ms[i] / launches[i] for up to cap kernels; returns count. */
int lzma_ctx_timings(lzma_ctx *ctx, const char **names, double *ms, int64_t *launches, int cap);
void lzma_ctx_reset_timings(lzma_ctx *ctx);
/* Host-side stalls of the context so far (cumulative; any pointer may be NULL):
 * allocations of its own device / pinned buffers (each one a hipFree + hipMalloc of a grown
 * buffer, hipMalloc of >100 GB workspaces costing tens of ms) with their bytes, and
 * whole-device synchronisations (hipDeviceSynchronize: a reallocation while a split encode is
 * in flight, an overflow-pool retry). A caller that reuses one batch layout must see none of
 * them after its first call: bench.py reports them for its sequential leg, and
 * tests/test_async_emulated.py asserts none after odd and even counts of split passes.
 * No reference counterpart (the Java encoder allocates per Create, Encoder.java:224-245). */
int lzma_ctx_stats(const lzma_ctx *ctx, uint64_t *allocations, uint64_t *alloc_bytes, uint64_t *device_syncs);

/* ---- encode -------------------------------------------------------------
 * Device-resident batch: stream i is d_in[h_offs[i] .. h_offs[i+1]).
 * Output region i is d_out[h_out_offs[i] .. h_out_offs[i+1]) (capacity,
 * use lzma_enc_bound); h_out_lens[i] receives the encoded length.
 * hip_stream: a hipStream_t or NULL. Returns LZMA_OK or an error code. */
int lzma_enc_batch_dev(lzma_ctx *ctx, const lzma_params *p,
                       const uint8_t *d_in, const uint64_t *h_offs, int nstreams,
                       uint8_t *d_out, const uint64_t *h_out_offs, uint64_t *h_out_lens,
                       void *hip_stream);
/* Gather stream i = d_src[h_src_offs[i] .. + h_lens[i]) to
 * d_dst[h_dst_offs[i] ..), h_dst_offs = exclusive prefix sum of h_lens
 * (nstreams+1 entries): packs capacity-layout encoder output. */
int lzma_pack_dev(lzma_ctx *ctx, const uint8_t *d_src, const uint64_t *h_src_offs, const uint64_t *h_lens,
                  int nstreams, uint8_t *d_dst, const uint64_t *h_dst_offs, void *hip_stream);
/* The same encode in three calls, for a caller that pipelines batches: the range
 * coder of one batch runs on the context's own coder stream while the next batch's
 * match finder runs on the caller's stream, and the next batch's walk on the
 * context's walk stream beside this batch's parser.
 *   lzma_enc_stage_dev: stages the batch (arguments as lzma_enc_batch_dev; d_in and
 *     d_out must stay valid until _wait) and enqueues its match finder's keys, sorts
 *     and chain lists on hip_stream. At most two batches are staged at once; a second
 *     one's match finder runs after the first one's walk. A batch staged alone on a
 *     context without a parse fence also gets its walk enqueued, whose grid is sized by
 *     a host read of the chain count: the call then waits for the work ahead on
 *     hip_stream and the sorts (not for the walk). Otherwise it returns without waiting.
 *   lzma_enc_parse_dev_async: for the oldest staged batch: the walk if not enqueued yet
 *     (it reads the chain count back), waits for the walk's verdict, then enqueues the
 *     parser on hip_stream (after the parse fence's decode, if any) and the range coder
 *     on the coder stream; then, if a second batch is staged, waits for its chain count
 *     and enqueues its walk on the walk stream (beside this parser); returns without
 *     waiting for the parser, the coder or that walk.
 *   lzma_enc_parse_dev_wait: waits for the oldest coder in flight; h_out_lens as
 *     lzma_enc_batch_dev for that batch.
 * One pass per batch: at most 16384 streams and lzma_ctx_set_batch_bytes of input
 * (LZMA_E_PARAM otherwise). At most two batches staged and two coders in flight (each
 * staged batch and each coder holds one of the context's two live slots); a third
 * stage or a parse_async with two coders in flight returns LZMA_E_PARAM, and consumes
 * nothing; any other failure of parse_async (never LZMA_E_PARAM once the oldest batch is
 * consumed) drops every staged batch. Without a parse fence, the round-4 order (stage A,
 * parse_async A, stage B, wait A) blocks the host in stage B until parser A has finished
 * (B is staged alone, so its walk is enqueued there, sized by a host read of its chain
 * count behind parser A on hip_stream): stage B before parse_async A to keep the overlap. Pipelined orders: stage k + 1, parse_async k,
 * wait k (with a parse fence); or stage 0, stage 1, parse_async 0, stage 2, then per k:
 * parse_async k + 1, stage k + 3, wait k (without one: parser k + 1 is enqueued while
 * coder k may still run, and batch k + 2's walk runs beside parser k + 1). While a batch is staged or its coder is in flight, the context's other
 * encode, decode and pack entry points return LZMA_E_PARAM. Reference: Encoder.Code
 * (Encoder.java:1064-1077), as for lzma_enc_batch_dev; the bytes are the same. */
int lzma_enc_stage_dev(lzma_ctx *ctx, const lzma_params *p,
                       const uint8_t *d_in, const uint64_t *h_offs, int nstreams,
                       uint8_t *d_out, const uint64_t *h_out_offs, void *hip_stream);
int lzma_enc_parse_dev_async(lzma_ctx *ctx, void *hip_stream);
int lzma_enc_parse_dev_wait(lzma_ctx *ctx, uint64_t *h_out_lens);
/* Host buffers: out is packed, out_offs[nstreams+1] receives the layout. */
int lzma_enc_batch(lzma_ctx *ctx, const lzma_params *p,
                   const uint8_t *in, const uint64_t *offs, int nstreams,
                   uint8_t *out, uint64_t out_cap, uint64_t *out_offs);
/* One stream: Encoder.Code(in, out, -1, -1, null).
 * Stream length: every stream must be shorter than 2^31 bytes (LZMA_E_PARAM
 * otherwise). This is an API departure from Encoder.Code, which accepts any
 * length and renormalises positions at 2^30 - 1 (BinTree.java:19, 88-90,
 * 358-375) without changing any output bit: the device keeps 32-bit positions
 * and about 100 bytes of workspace per input byte.
 * Longer inputs are encoded as independent streams. */
int lzma_encode(lzma_ctx *ctx, const lzma_params *p, const uint8_t *in, uint64_t n,
                uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* ---- the sliced encode: ONE long stream in bounded device launches ------
 * Encoder.Code (Encoder.java:1064-1077) over one stream, the parse and range coder run a
 * slice at a time: every launch stops at the first CodeOneBlock boundary
 * (Encoder.java:843-936; no look-ahead pending) past its stop position, with the
 * encoder's state (models, price tables and their refresh countdowns, reps, the range
 * coder's low / range / cache) kept in HBM for the next launch. The bytes are exactly
 * lzma_encode's. What it is for: a single serial parse of a 1 GiB stream is one ~30-minute
 * kernel; slices bound every launch (watchdogs, preemption), report progress between them
 * (ICodeProgress.SetProgress, Encoder.java:1070-1072, at block granularity instead of once
 * at the end), and checkpoint to the host so another process can finish the stream.
 *   lzma_enc_session_begin: d_in[0 .. n) device-resident, n < 2^31; d_out of at least
 *     lzma_enc_bound(n) bytes, both valid until _end. Runs the match finder over the whole
 *     stream (it is a pure function of the input, so a restored session recomputes it).
 *     While the session is open the context's other encode / decode / pack entry points
 *     return LZMA_E_PARAM.
 *   lzma_enc_session_step: parses and codes at least `bytes` more input (a slice ends at
 *     the next block boundary, within 4 KiB + 273 bytes past that) and appends the slice's
 *     final output bytes at d_out[*out_len ..]; *in_pos = input consumed, *out_len = output
 *     bytes final so far, *done = 1 once the stream is flushed (then a no-op).
 *   lzma_enc_session_save: the state after the last step as a blob (blob NULL: *len =
 *     the size needed): parameters, positions, coder state, the parser state (~6 KiB plus
 *     the literal coders, 12 KiB at lc 3).
 *   lzma_enc_session_restore: on a fresh session over the same input and parameters
 *     (before its first step): go on from the blob; the caller keeps the first *out_len
 *     output bytes (they are final) and the session writes after them.
 * No reference counterpart beyond Encoder.Code itself (the Java encoder keeps its state
 * in the Encoder instance between CodeOneBlock calls, Encoder.java:843-936). */
typedef struct lzma_enc_session lzma_enc_session;
int lzma_enc_session_begin(lzma_ctx *ctx, const lzma_params *p, const uint8_t *d_in, uint64_t n,
                           uint8_t *d_out, uint64_t out_cap, void *hip_stream, lzma_enc_session **out);
int lzma_enc_session_step(lzma_enc_session *s, uint64_t bytes, uint64_t *in_pos, uint64_t *out_len, int *done);
int lzma_enc_session_save(const lzma_enc_session *s, uint8_t *blob, uint64_t cap, uint64_t *len);
int lzma_enc_session_restore(lzma_enc_session *s, const uint8_t *blob, uint64_t len);
void lzma_enc_session_end(lzma_enc_session *s);
/* Host-buffer form (the JNI drop-in's Encoder.Code with an ICodeProgress): the input is
 * copied to the context's device staging; after each step, lzma_enc_session_output copies
 * final output bytes [from, from + len), from + len <= *out_len, to the host, so the caller
 * can write them to its OutputStream and call SetProgress(in_pos, out_len) slice by slice. */
int lzma_enc_session_begin_host(lzma_ctx *ctx, const lzma_params *p, const uint8_t *in, uint64_t n,
                                lzma_enc_session **out);
int lzma_enc_session_output(const lzma_enc_session *s, uint64_t from, uint8_t *dst, uint64_t len);

/* ---- decode -------------------------------------------------------------
 * props: the 5 property bytes (Decoder.SetDecoderProperties).
 * h_out_sizes[i] = outSize of Decoder.Code (-1 => until end marker).
 * h_status[i] = LZMA_OK, LZMA_E_DATA (Decoder.Code false) or LZMA_E_OVERFLOW.
 * h_out_lens[i] = bytes decoded. As in Decoder.Code, a match may run past
 * outSize (CopyBlock copies whole matches, OutWindow.java:53-67), so a region
 * needs outSize + 273 bytes of capacity to never report LZMA_E_OVERFLOW.
 * On LZMA_E_DATA the region holds every byte decoded before the corrupt
 * symbol; the reference's OutputStream has by then received only the whole
 * windows OutWindow flushed (OutWindow.java:63-73, window = max(dict, 4096),
 * Decoder.java:167), i.e. the first floor(len / window) * window bytes.
 * lzma_visible_on_error() gives that prefix length; the drop-ins write it.
 * Input is consumed whole: the reference's RangeDecoder reads its stream
 * lazily (RangeDecoder.java:19-25) and leaves bytes past the stream unread,
 * a departure the drop-in handles with mark/reset where the stream allows. */
uint64_t lzma_visible_on_error(uint32_t dict_size, uint64_t decoded_len);
int lzma_dec_batch_dev(lzma_ctx *ctx, const uint8_t props[5],
                       const uint8_t *d_in, const uint64_t *h_in_offs, int nstreams,
                       const int64_t *h_out_sizes,
                       uint8_t *d_out, const uint64_t *h_out_offs, uint64_t *h_out_lens,
                       int32_t *h_status, void *hip_stream);
/* Pipelined form of lzma_dec_batch_dev (no Java counterpart: a batch
 * scheduling aid). _async enqueues the decode on hip_stream and returns at
 * once (the host arrays are copied into the context's pinned staging first);
 * _wait blocks until it is done and writes h_out_lens / h_status (either may
 * be NULL). One decode may be in flight per context, and the context runs
 * nothing else until _wait (every other entry point returns LZMA_E_PARAM).
 * Another context may encode meanwhile, on another HIP stream. */
int lzma_dec_batch_dev_async(lzma_ctx *ctx, const uint8_t props[5],
                             const uint8_t *d_in, const uint64_t *h_in_offs, int nstreams,
                             const int64_t *h_out_sizes, uint8_t *d_out, const uint64_t *h_out_offs,
                             void *hip_stream);
int lzma_dec_batch_dev_wait(lzma_ctx *ctx, uint64_t *h_out_lens, int32_t *h_status);
/* Encode passes on ctx launch their parser only after dec_ctx's decode in
 * flight (if any) has finished: the parser wants every stream resident from
 * its start, so a concurrent decode may share the match finder's time but not
 * the parse's. NULL clears the fence; destroying dec_ctx clears it too. */
int lzma_ctx_set_parse_fence(lzma_ctx *ctx, const lzma_ctx *dec_ctx);
int lzma_dec_batch(lzma_ctx *ctx, const uint8_t props[5],
                   const uint8_t *in, const uint64_t *in_offs, int nstreams,
                   const int64_t *out_sizes, uint8_t *out, const uint64_t *out_offs,
                   uint64_t *out_lens, int32_t *status);
int lzma_decode(lzma_ctx *ctx, const uint8_t props[5], const uint8_t *in, uint64_t n,
                int64_t out_size, uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* ---- several devices from one process (SURVEY 8(b) `device_mask`) --------
 * A multi-device context holds one lzma_ctx per device whose bit is set in
 * device_mask. The batch entry points deal the streams round-robin over those
 * devices (the j-th selected device takes streams j, j+D, j+2D, ...: SURVEY
 * 8(e)'s {i : i mod G = r}), run each device from its own host thread, and
 * return the outputs in stream order, with the same layout and meaning as
 * lzma_enc_batch / lzma_dec_batch. */
typedef struct lzma_mctx lzma_mctx;
int lzma_mctx_create(uint32_t device_mask, lzma_mctx **out);
void lzma_mctx_destroy(lzma_mctx *m);
const char *lzma_mctx_last_error(const lzma_mctx *m);
int lzma_mctx_devices(const lzma_mctx *m);
/* lzma_ctx_set_batch_bytes / lzma_ctx_set_timing applied to every device's context. */
int lzma_mctx_set_batch_bytes(lzma_mctx *m, uint64_t bytes);
int lzma_mctx_set_timing(lzma_mctx *m, int on);
int lzma_enc_batch_multi(lzma_mctx *m, const lzma_params *p, const uint8_t *in, const uint64_t *offs, int nstreams,
                         uint8_t *out, uint64_t out_cap, uint64_t *out_offs);
int lzma_dec_batch_multi(lzma_mctx *m, const uint8_t props[5], const uint8_t *in, const uint64_t *in_offs,
                         int nstreams, const int64_t *out_sizes, uint8_t *out, const uint64_t *out_offs,
                         uint64_t *out_lens, int32_t *status);

/* ---- instrumented mode --------------------------------------
 * The GPU match finder's per-position output for a batch of streams, as
 * BinTree.GetMatches (BinTree.java:152-273) returns it at every position plus
 * the ReadMatchDistances extension of the longest pair (Encoder.java:275-287):
 * counts[g] pairs and main_len[g] for every input byte g (total = offs[n] -
 * offs[0]), the pairs of all positions in order into lens/dists (at most
 * cap; *total_pairs gets the full count, LZMA_E_OVERFLOW if it exceeds cap).
 * A diagnostic for parity tests: the encoder consumes the same arrays. */
int lzma_match_lists(lzma_ctx *ctx, const lzma_params *p, const uint8_t *in, const uint64_t *offs, int nstreams,
                     uint32_t *counts, uint32_t *main_len, uint32_t *lens, uint32_t *dists, uint64_t cap,
                     uint64_t *total_pairs);

/* ---- synthetic inputs (bench / tests) ----------------------------------- */
/* LzmaBench.CBenchRandomGenerator.Generate (LzmaBench.java:104-127). */
void lzma_bench_generate(uint8_t *buf, uint64_t size);
/* RND: SplitMix64 outputs, little-endian. */
void lzma_rnd_generate(uint8_t *buf, uint64_t size, uint64_t seed);
/* TEXT ("enwik9-shaped"): Zipf(1.1) words over a fixed
 * 50k-word synthetic vocabulary with wiki-style markup about every 200 words. */
void lzma_text_generate(uint8_t *buf, uint64_t size, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* LZMA_MI355X_H */
