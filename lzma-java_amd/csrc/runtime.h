// runtime.h -- device context, workspace arena, per-kernel HIP-event timing and
// the argument blocks shared by the kernels and the host orchestration.
#pragma once

#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

#include <atomic>
#include <map>
#include <thread>
#include <string>
#include <vector>

#include "lzma_common.h"

namespace lzg {

// Experiment switches (A/B timing runs: walk subsets, thresholds, off-by-default kernel
// variants) read the environment only in the experiment build (`make exp`, -DLZG_EXPERIMENT).
// The product library ignores them, so its output never depends on the caller's environment.
static inline const char* exp_env(const char* name) {
#ifdef LZG_EXPERIMENT
    return getenv(name);
#else
    (void)name;
    return nullptr;
#endif
}


struct MfArgs {
    uint32_t fb, min_match_check, hash_mask, hash_bits, cut_value, direct_bytes;
    uint32_t rec_vecs;            // 16-byte vectors per match-list record
    uint64_t cyc_size;
    uint64_t* k4;
    uint32_t *k3, *k2;            // (stream << 16 | hash3), (stream << 10 | hash2): < 2^30 for <= 16384 streams
    uint32_t* prev3;              // hash3 "last occurrence" by position (mf_prev_kernel)
    v4u32* mrec;                  // per-position match-list records (lzma_common.h store_rec)
    uint32_t walk_lo, walk_hi;    // experiment hook (LZG_WALK_ONLY): walk only chains of length in [lo, hi]
    uint64_t total;               // positions of the pass (every chain, sorted index and position is below it)
    int nstreams;
};

struct MfBuffers {
    uint64_t *k4, *ks;            // k4's memory holds the long-chain lists after the hash4 sort
    uint32_t *k3, *k2;            // also the walk-order keys (k2) and their sorted copy (k3)
    uint32_t *vs, *prev3;
    uint32_t *chain_start, *chain_len, *chain_order;
    uint32_t* cls;                // long chains per length class [32], the scatter cursors [32], the long count [1]
    uint64_t* son;                // walk tree nodes (mf.hip WNode, 32 B per position: links + 16-byte prefix);
                                  // before the walk, the sorts' ping-pong buffers
    uint32_t* hist;               // sort.hip digit histograms, [nstreams][4][256]
    uint64_t* seg_end;            // per stream: the end of its chain list (mf_chains_kernel)
    uint64_t* chain_offs;         // per stream: where its chains start in the compacted walk order; [nstreams] = chains
    v4u32* pairs;                 // per-position match-list records: inline pairs + info (lzma_common.h)
    uint32_t* ovf_off;
    void* ovf;
    uint64_t ovf_cap;
    unsigned long long* ovf_used;
    int* err;
};

struct Ctx;

struct TimedLaunch {
    Ctx* ctx;
    const char* name;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    TimedLaunch(Ctx* c, const char* n, hipStream_t s);
    ~TimedLaunch();
};

// Handle tags: every C entry point checks the tag of the handle it is given, so an
// lzma_mctx* (multi.hip) passed where an lzma_ctx* is expected is rejected with
// LZMA_E_PARAM instead of being written through.
constexpr uint32_t kCtxMagic = 0x58435A4Cu;    // "LZCX"
constexpr uint32_t kMctxMagic = 0x584D5A4Cu;   // "LZMX" (multi.hip)

// A device buffer that grows on demand and is kept for the context's lifetime, so
// repeated host-buffer calls (the JNI single-stream path) allocate nothing per call.
struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    uint64_t allocs = 0, alloc_bytes = 0;   // reallocations (lzma_ctx_stats)
    bool ensure(size_t want) {
        if (want <= n) return true;
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
        allocs++;
        alloc_bytes += want;
        if (hipMalloc(&p, want) != hipSuccess) return false;
        n = want;
        return true;
    }
    void release() {
        if (p) hipFree(p);
        p = nullptr;
        n = 0;
    }
    template <typename T> T* as() const { return (T*)p; }
};

// Pinned host staging, grown on demand. Copies between the host and the device
// go through it: a copy from pageable memory may wait for the whole device (an
// encode on one HIP stream would then wait for a decode running on another).
struct HostBuf {
    void* p = nullptr;
    size_t n = 0;
    uint64_t allocs = 0, alloc_bytes = 0;   // reallocations (lzma_ctx_stats)
    bool ensure(size_t want) {
        if (want <= n) return true;
        if (p) hipHostFree(p);
        p = nullptr;
        n = 0;
        allocs++;
        alloc_bytes += want;
        if (hipHostMalloc(&p, want, 0) != hipSuccess) return false;
        n = want;
        return true;
    }
    void release() {
        if (p) hipHostFree(p);
        p = nullptr;
        n = 0;
    }
    template <typename T> T* as(size_t byte_off = 0) const { return (T*)((uint8_t*)p + byte_off); }
};

struct EncPass;   // runtime.hip: one encode pass in pieces

struct Ctx {
    uint32_t magic = kCtxMagic;   // first member: see kCtxMagic
    int device = 0;
    // host-buffer entry points (lzma_enc_batch, lzma_dec_batch, lzma_match_lists): staging in HBM
    DevBuf io_in, io_out, io_pack, io_offs;
    HostBuf pin;        // encode-pass and pack staging (offsets, order, lengths, status)
    HostBuf pin_mf;     // the match finder's chain-count and walk-verdict readback, 32 bytes per slot
    std::string err;
    bool debug = getenv("LZMA_MI355X_DEBUG") != nullptr;   // phase trace on stderr (synchronises)
    uint64_t batch_bytes = 512ull << 20;
    // persistent workspace arena (grown, never shrunk): the match finder's scratch, the
    // parser's spill scratch, the decoder's and pack's workspace
    uint8_t* arena = nullptr;
    size_t arena_size = 0;
    // an encode pass's buffers that live from its staging to its parse (input copy, pass
    // arrays, match lists, overflow pool): slot 0 for the synchronous form, slots 0 / 1
    // alternating for the split form, so one pass's walk can run beside the other's parse
    DevBuf live[2];
    uint8_t* tmp = nullptr;     // cub temp storage
    size_t tmp_size = 0;
    uint64_t ovf_hint = 0;      // overflow pool slots per 1024 input bytes (0 = default; grows on retry)
    // asynchronous batch decode (lzma_dec_batch_dev_async / _wait): the per-stream
    // lengths and verdicts land in pinned host memory, `dec_done` marks the end
    uint64_t* dec_host = nullptr;    // pinned: offsets/sizes staging, then lens (n) + status (n / 2 words)
    size_t dec_host_words = 0;
    int dec_pending = 0;             // streams of the decode in flight (0 = none)
    hipEvent_t dec_done = nullptr;
    hipStream_t dec_stream = nullptr;
    // parse fence (lzma_ctx_set_parse_fence): an encode pass waits for this
    // context's decode in flight before it launches its parser
    const Ctx* fence = nullptr;
    // split encode (lzma_enc_stage_dev -> lzma_enc_parse_dev_async -> lzma_enc_parse_dev_wait):
    // the staged pass, and the range coder in flight on the context's coder stream
    // the staged passes (at most two: the older one's parse may run beside the newer one's
    // walk), oldest at split_head; split_state = how many are staged
    EncPass* split_pass[2] = {nullptr, nullptr};
    int split_head = 0;
    int split_state = 0;
    // range coders in flight (at most two, one per slot, oldest first): rc_pending = how many
    int rc_pending = 0;
    int rc_slot[2] = {0, 0}, rc_ns[2] = {0, 0};   // rc_slot: the coder set (coder_bind)
    hipEvent_t rc_done[2] = {nullptr, nullptr}, parse_done[2] = {nullptr, nullptr};
    hipEvent_t cnt_done[2] = {nullptr, nullptr};    // per slot: the chain count copied to the host
    hipEvent_t walk_done[2] = {nullptr, nullptr};   // per slot: the walk's verdict copied to the host
    hipEvent_t parse_start = nullptr;      // the split form: st has reached the parser (past the fence)
    hipStream_t rc_stream = nullptr;       // created on first use
    hipStream_t walk_stream = nullptr;     // a staged pass's walk beside the older pass's parse
    DevBuf split_recs[2], split_coder[2];  // per coder set: the coder records and per-stream arrays (apart from the arena)
    HostBuf pin_rc[2];                     // per slot: the coder's lengths and verdicts, written by the device
    // an open sliced encode (lzma_enc_session_*) holds the live slot and the arena: the
    // context's other encode, decode and pack entry points refuse while it is open
    struct EncSession* session = nullptr;
    // timing
    bool timing = false;
    struct Pending { std::string name; hipEvent_t a, b; };
    std::vector<Pending> pending;
    std::vector<hipEvent_t> free_events;
    struct Acc { double ms = 0; int64_t n = 0; };
    std::map<std::string, Acc> acc;

    // Host-side events that stall a pipelined caller (lzma_ctx_stats): allocations of the
    // context's own buffers (hipMalloc / hipHostMalloc after a hipFree of the smaller one) and
    // whole-device synchronisations. The DevBuf / HostBuf members count their own.
    uint64_t stat_allocs = 0, stat_alloc_bytes = 0, stat_device_syncs = 0;
    hipError_t device_sync() {
        stat_device_syncs++;
        return hipDeviceSynchronize();
    }
    void count_alloc(size_t n) {
        stat_allocs++;
        stat_alloc_bytes += n;
    }

    int fail(int code, const char* fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        return code;
    }
    void* scratch(size_t n) {
        if (n == 0) return tmp;
        if (n > tmp_size) {
            if (tmp) hipFree(tmp);
            tmp = nullptr;
            tmp_size = 0;
            count_alloc(n);
            if (hipMalloc(&tmp, n) != hipSuccess) return nullptr;
            tmp_size = n;
        }
        return tmp;
    }
    // literal-coder tables of the encoder and decoder: their own allocation, so the
    // per-stream tables sit in one compact region (few TLB pages) instead of at a
    // large stride inside the match-finder arena
    uint8_t* litbuf = nullptr;
    size_t litbuf_size = 0;
    bool ensure_litbuf(size_t n) {
        if (n <= litbuf_size) return true;
        if (litbuf) hipFree(litbuf);
        litbuf = nullptr;
        litbuf_size = 0;
        count_alloc(n);
        if (hipMalloc(&litbuf, n) != hipSuccess) return false;
        litbuf_size = n;
        return true;
    }
    bool ensure_arena(size_t n) {
        if (n <= arena_size) return true;
        if (arena) hipFree(arena);
        arena = nullptr;
        arena_size = 0;
        count_alloc(n);
        if (hipMalloc(&arena, n) != hipSuccess) return false;
        arena_size = n;
        return true;
    }
    hipEvent_t get_event() {
        if (!free_events.empty()) { hipEvent_t e = free_events.back(); free_events.pop_back(); return e; }
        hipEvent_t e;
        hipEventCreate(&e);
        return e;
    }
    void resolve_timings() {
        for (auto& p : pending) {
            hipEventSynchronize(p.b);
            float ms = 0;
            hipEventElapsedTime(&ms, p.a, p.b);
            Acc& a = acc[p.name];
            a.ms += ms;
            a.n += 1;
            free_events.push_back(p.a);
            free_events.push_back(p.b);
        }
        pending.clear();
    }
};

// debug trace: synchronise the stream and print a phase marker
#define LZG_TRACE(ctx, st, ...)                                                     \
    do {                                                                            \
        if ((ctx)->debug) {                                                         \
            hipError_t e_ = hipStreamSynchronize(st);                               \
            fprintf(stderr, "[lzma-mi355x] ");                                      \
            fprintf(stderr, __VA_ARGS__);                                           \
            fprintf(stderr, " (%s)\n", hipGetErrorString(e_));                      \
            fflush(stderr);                                                         \
        }                                                                           \
    } while (0)

// Debug-only live view of a running kernel: the kernel stores checkpoints into
// host-mapped memory; a host thread prints them until stop().
struct DebugWatch {
    uint32_t* host = nullptr;
    uint32_t* dev = nullptr;
    std::atomic<bool> run{false};
    std::thread th;
    void start(int words) {
        if (hipHostMalloc((void**)&host, words * 4, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) { host = nullptr; return; }
        memset(host, 0, words * 4);
        hipHostGetDevicePointer((void**)&dev, host, 0);
        run = true;
        th = std::thread([this, words]() {
            std::vector<uint32_t> last(words, 0);
            while (run) {
                std::this_thread::sleep_for(std::chrono::milliseconds(500));
                bool ch = false;
                for (int i = 0; i < words; i++) if (((volatile uint32_t*)host)[i] != last[i]) ch = true;
                if (!ch) continue;
                fprintf(stderr, "[lzma-mi355x dbg]");
                for (int i = 0; i < words; i++) { last[i] = ((volatile uint32_t*)host)[i]; fprintf(stderr, " %u", last[i]); }
                fprintf(stderr, "\n");
                fflush(stderr);
            }
        });
    }
    void stop() {
        if (!host) return;
        run = false;
        th.join();
        hipHostFree(host);
        host = dev = nullptr;
    }
};

inline TimedLaunch::TimedLaunch(Ctx* c, const char* n, hipStream_t s) : ctx(c), name(n), st(s) {
    if (ctx->timing) { a = ctx->get_event(); b = ctx->get_event(); hipEventRecord(a, st); }
}
inline TimedLaunch::~TimedLaunch() {
    if (ctx->timing) { hipEventRecord(b, st); ctx->pending.push_back({name, a, b}); }
}

// bump carve of a device arena
struct Carver {
    uint8_t* base;
    size_t off = 0;
    explicit Carver(uint8_t* b) : base(b) {}
    template <typename T> T* take(size_t count) {
        off = (off + 255) & ~(size_t)255;
        T* p = (T*)(base + off);
        off += count * sizeof(T);
        return p;
    }
};

__global__ void iota_kernel(uint32_t* out, uint64_t n);

// overflow pool slot: pairs beyond the inline ones of one position (at most
// fb - 1 pairs per position: lengths 2..fb, strictly increasing)
__host__ __device__ inline uint32_t ovf_stride(uint32_t fb) { return fb > (uint32_t)kInlinePairs + 1 ? fb - 1 - kInlinePairs : 1u; }

int mf_front(Ctx* ctx, const Derived& d, const uint8_t* in, const uint64_t* d_offs, int nstreams, uint64_t total,
             bool wide_pairs, MfBuffers& w, hipStream_t st);
int mf_back(Ctx* ctx, const Derived& d, const uint8_t* in, const uint64_t* d_offs, int nstreams, uint64_t total,
            bool wide_pairs, MfBuffers& w, hipStream_t st);
// mf_back in pieces, per pinned slot (0 / 1): the chain count's copy to the host enqueued
// on the match finder's stream (cnt_done[slot] behind it); the walk, sized from that
// count (the host waits for cnt_done[slot] only), and its verdict's copy enqueued on st
// (which may be another stream: the split encode runs a staged pass's walk beside the
// older pass's parse); the verdict once st has passed that copy
int mf_count_enqueue(Ctx* ctx, const MfBuffers& w, int nstreams, hipStream_t st, int slot);
int mf_walk_launch(Ctx* ctx, const Derived& d, const uint8_t* in, const uint64_t* d_offs, int nstreams, uint64_t total,
                   bool wide_pairs, MfBuffers& w, hipStream_t st, int slot);
int mf_walk_result(Ctx* ctx, int slot);
// sort.hip: stable per-stream radix sort by the low end_bit key bits; the `hist` words it
// needs for n items in nstreams segments
size_t sort_hist_words(uint64_t n, int nstreams);
// sort.hip: stable per-stream radix sort by the low end_bit key bits
int seg_radix_sort(Ctx* ctx, bool key64, const void* kin, const uint32_t* vin, void* kout, uint32_t* vout,
                   uint64_t* tmp_a, uint64_t* tmp_b, uint32_t* hist, uint64_t n, const uint64_t* d_offs, int nstreams,
                   int end_bit, hipStream_t st, const uint64_t* d_ends = nullptr, const uint64_t* d_dofs = nullptr);

struct EncArgs {
    const uint8_t* in;            // padded batch copy
    const uint64_t* offs;         // stream offsets (nstreams+1)
    const uint32_t* order;        // processing order (longest first)
    int nstreams;
    unsigned int* next;           // work-queue counter
    const v4u32* pairs;           // per-position match-list records (lzma_common.h store_rec)
    const uint32_t* ovf_off;
    const void* ovf;
    uint16_t* recs;               // coder records (rc.hip), per stream at rec_offs[s]
    const uint64_t* rec_offs;     // record capacity layout (nstreams+1), multiples of 64 records
    uint64_t* rec_lens;           // records emitted per stream
    uint64_t* out_lens;           // diagnostic (reason << 32 | position) of streams that tripped a check
    int32_t* status;
    uint8_t* scratch;             // per-block global scratch (_optimum spill)
    uint64_t scratch_stride;
    uint8_t* lit_scratch;         // per-block literal coders (when not in LDS), Ctx::litbuf
    uint64_t lit_stride;
    uint32_t fb, lc, lp, pb, eos, dist_table_size, len_table_size;
    uint32_t lit_in_lds;
    uint32_t pair_bytes;          // 4 (u32 packed pairs) or 8 (u64, streams >= 8 MiB)
    // the sliced encode (lzma_enc_session_*, the LZG_ENC_SLICED kernels): per-stream parser state
    // in HBM (enc.hip slice_layout), a parse that stops at the first CodeOneBlock boundary
    // (additional_offset == 0) with now_pos >= slice_stop, or resumes from the saved state
    uint8_t* slice_state;
    uint64_t slice_stride;
    uint32_t slice_stop, slice_resume;
    uint32_t* dbg;                // debug checkpoints (host-mapped, LZMA_MI355X_DEBUG only) or null
    uint64_t* prof;               // phase cycles [nstreams][kProfSlots] (LZG_PROF builds) or null
};

// encoder phase profile slots (LZG_PROF builds)
enum { PF_TOTAL, PF_GETOPT, PF_MATCHES, PF_REPLEN, PF_TWOLEN, PF_LIT, PF_RELAX, PF_TWOREL, PF_STATE, PF_BACK,
       PF_ENCODE, PF_TABLES, PF_NOPT, PF_NPOS, PF_NSPILL, PF_NOVF, PF_NTWO, PF_T0, PF_T1, PF_HWID, kProfSlots };

int launch_encoder(Ctx* ctx, const EncArgs& a, bool wide_pairs, int grid, hipStream_t st);
// enc_slice.hip: the same parser compiled with LZG_ENC_SLICED (stop / resume at CodeOneBlock
// boundaries); the per-stream state size for these parameters
int launch_encoder_sliced(Ctx* ctx, const EncArgs& a, bool wide_pairs, int grid, hipStream_t st);
size_t enc_slice_state_bytes(const Derived& d);
// scalar words at the front of a stream's slice state (enc.hip), readable by the host
enum { SS_MAGIC, SS_NOW_POS, SS_DONE, SS_STATE, SS_PREV_BYTE, SS_REP0, SS_REP1, SS_REP2, SS_REP3, SS_MATCH_PRICE_COUNT,
       SS_ALIGN_PRICE_COUNT, SS_WORDS = 16 };
constexpr uint32_t kSliceMagic = 0x534C5A4Cu;   // "LZLS"

// rc.hip: the range coder over the parser's records, one lane per stream
struct RcArgs {
    uint16_t* recs;               // read, then reused as each stream's output staging
    const uint64_t* rec_offs;
    const uint64_t* rec_lens;
    const uint32_t* order;        // longest first: the lanes of a wave get similar record counts
    int nstreams;
    int32_t* status;              // in: the parser's verdict; out: LZMA_E_OVERFLOW when the output does not fit
    uint8_t* out;
    const uint64_t* out_offs;     // output capacity layout (nstreams+1)
    uint64_t* out_lens;
    uint32_t* seg;                // [nstreams][kRcSegs][kRcSegWords]: start range, bytes, lo, carry, cache, cache size,
                                  // end range
    // The sliced encode (lzma_enc_session_*): a stream's records arrive slice by slice and the
    // coder carries its state from one slice to the next. sliced: segment 0 starts from
    // init_state (null: Init), the segments are cut so the last non-empty one holds the coder's
    // end state (rc_seglen), and without `flush` the unfinished digits stay out of the output
    // and the end state goes to end_state. State words: range, lo, carry, cache, cache size.
    uint32_t sliced, flush;
    const uint32_t* init_state;   // [nstreams][kRcStateWords] or null
    uint32_t* end_state;          // [nstreams][kRcStateWords] or null
};
constexpr int kRcStateWords = 8;
constexpr int kRcSegs = 16;       // coder segments per stream (rc.hip)
constexpr int kRcSegWords = 8;
int launch_rc(Ctx* ctx, const RcArgs& a, hipStream_t st);
// records one stream of n bytes can need: <= 21 per byte (a length-2 match: isMatch, isRep,
// 4 length bits, 6 slot bits, 30 footer bits), the end marker (42) and the first literal
__host__ __device__ inline uint64_t rc_record_bound(uint64_t n) { return (24 * n + 64 + 63) & ~(uint64_t)63; }
uint32_t enc_lit_in_lds(const Derived& d, int nstreams);
size_t enc_scratch_per_block(const Derived& d);
size_t enc_lit_bytes(const Derived& d);

struct DecArgs {
    const uint8_t* in;
    const uint64_t* in_offs;
    const int64_t* out_sizes;
    uint8_t* out;
    const uint64_t* out_offs;
    uint64_t* out_lens;
    int32_t* status;
    const uint32_t* order;
    int nstreams;
    unsigned int* next;
    uint8_t* scratch;             // per-block literal probs when they do not fit LDS
    uint64_t scratch_stride;
    uint32_t lc, lp, pb, dict_check, lit_in_lds;
};

int launch_decoder(Ctx* ctx, const DecArgs& a, int grid, hipStream_t st);
int dec_grid(uint32_t lc, uint32_t lp, uint32_t lit_in_lds, int nstreams);
int enc_grid(const Derived& d, int nstreams);
size_t enc_lds_bytes(const EncArgs& a);
size_t dec_scratch_per_block(uint32_t lc, uint32_t lp);

}  // namespace lzg

struct lzma_ctx : lzg::Ctx {};
