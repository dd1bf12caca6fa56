// runtime.hip -- host orchestration and the C ABI (include/lzma_mi355x.h).
//
// Encode of a batch of independent streams = one or more device passes, each
// bounded by Ctx::batch_bytes of input:
//   pad-copy input -> phase 1 match finder (mf.hip) -> phase 2 parser +
//   range coder (enc.hip), all on one HIP stream; the host only reads back
//   the per-stream lengths/status. Decode = dec.hip on the same model.
// There is no CPU fallback: without a HIP device every entry point that
// would compute returns LZMA_E_NODEVICE.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <numeric>
#include <set>
#include <vector>

#include "lzma_common.h"
#include "runtime.h"

namespace lzg {

__global__ void iota_kernel(uint32_t* out, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = (uint32_t)i;
}

// gather per-stream outputs into a packed buffer: block per stream
__global__ void pack_kernel(const uint8_t* __restrict__ src, const uint64_t* __restrict__ src_offs,
                            const uint64_t* __restrict__ dst_offs, uint8_t* __restrict__ dst, int nstreams) {
    for (int s = blockIdx.x; s < nstreams; s += gridDim.x) {
        uint64_t a = src_offs[s], o = dst_offs[s], len = dst_offs[s + 1] - o;
        for (uint64_t i = threadIdx.x; i < len; i += blockDim.x) dst[o + i] = src[a + i];
    }
}

static bool ok_ctx(const Ctx* c) { return c && c->magic == kCtxMagic; }

// Live contexts: lzma_ctx_destroy clears every parse fence that names the context
// being destroyed, so a fence never points at freed memory.
static std::mutex g_ctx_lock;
static std::set<Ctx*> g_live_ctx;

static int check_device(Ctx* ctx) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return ctx ? ctx->fail(LZMA_E_NODEVICE, "no HIP device (the MI355X path has no CPU fallback)") : LZMA_E_NODEVICE;
    return LZMA_OK;
}

#define HIPCHK(x)                                                                      \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)

#ifdef LZG_PROF
// Per-phase s_memtime cycles summed over the pass's streams (stderr).
static void report_profile(const uint64_t* d_prof, int ns, uint64_t total, hipStream_t st) {
    std::vector<uint64_t> h((size_t)ns * kProfSlots);
    hipMemcpyAsync(h.data(), d_prof, h.size() * 8, hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    static const char* names[kProfSlots] = {"total", "get_optimum", "match_lists", "rep_len", "two_step_len", "lit_price",
                                            "relax", "two_step_relax", "state", "backward", "encode", "tables",
                                            "n_getopt", "n_positions", "n_spill_steps", "n_ovf_lists",
                                            "n_two_step", "t0", "t1", "hwid"};
    double sum[kProfSlots] = {0};
    uint64_t mx = 0;
    for (int i = 0; i < ns; i++) {
        for (int k = 0; k < kProfSlots; k++) sum[k] += (double)h[(size_t)i * kProfSlots + k];
        mx = std::max(mx, h[(size_t)i * kProfSlots]);
    }
    fprintf(stderr, "[lzg prof] %d streams, %llu bytes, max stream cycles %llu\n", ns, (unsigned long long)total,
            (unsigned long long)mx);
    for (int k = 0; k < PF_T0; k++)
        fprintf(stderr, "[lzg prof] %-15s %16.0f  %8.1f per byte  %5.1f%%\n", names[k], sum[k], sum[k] / (double)total,
                k < PF_NOPT ? 100.0 * sum[k] / std::max(sum[0], 1.0) : 0.0);
    // placement: wall-clock start/end per stream, grouped by CU (xcc, se, sh, cu)
    if (getenv("LZG_PROF_DUMP")) {
        FILE* f = fopen(getenv("LZG_PROF_DUMP"), "w");
        if (f) {
            fprintf(f, "stream,t0,t1,cycles,npos,hwid,xcc\n");
            for (int i = 0; i < ns; i++) {
                const uint64_t* r = &h[(size_t)i * kProfSlots];
                fprintf(f, "%d,%llu,%llu,%llu,%llu,%u,%u\n", i, (unsigned long long)r[PF_T0], (unsigned long long)r[PF_T1],
                        (unsigned long long)r[PF_TOTAL], (unsigned long long)r[PF_NPOS], (unsigned)(r[PF_HWID] & 0xFFFFFFFFu),
                        (unsigned)(r[PF_HWID] >> 32));
            }
            fclose(f);
        }
    }
}
#endif

// Parser scratch is ~160 KiB per stream (one workgroup each): cap a pass at
// 16384 streams (~2.6 GB).
constexpr int kMaxStreamsPerPass = 16384;

// Host copies of the match finder's per-position output (the instrumented
// mode of SURVEY 7.1: lzma_match_lists diffs them against the oracle).
struct MatchDump {
    std::vector<uint32_t> ovf_off;
    std::vector<uint8_t> recs, ovf;
    bool wide = false;
    uint32_t stride = 0;
};

// One encode pass over streams [s0, s1) of a batch, in pieces: plan (host arrays),
// carve (the arena layout), stage (input and offsets to the device), the match
// finder's front (keys, sorts, chain lists: enqueued only) and back (the walk; reads
// the chain count and the walk's verdict back), the parser, the range coder. The
// synchronous entry points run them back to back on one HIP stream (encode_pass);
// the split form (lzma_enc_stage_dev / lzma_enc_parse_dev_async / _wait) runs the
// range coder on the context's coder stream, out of buffers no later pass touches
// while it runs, so a pipelined caller overlaps it with the next batch's match finder.
struct EncPass {
    Derived d{};
    const uint8_t* d_in = nullptr;
    uint8_t* d_out = nullptr;
    int ns = 0;
    uint64_t in0 = 0, total = 0;
    bool wide = false, split = false;
    int slot = 0;                 // live buffers, pinned words and events of ctx (split form: 0 / 1)
    const uint8_t* carved_arena = nullptr;   // ctx->arena when the shared buffers were carved
    int walk_state = 0;           // the split form: 0 the walk not enqueued, 1 enqueued (walk_done[slot] behind it)
    size_t psz = 4;
    std::vector<uint64_t> offs, oofs, rofs;
    std::vector<uint32_t> order;
    int grid = 0;
    size_t scr = 0;
    uint64_t stride = 0, slots_per_k = 64, ovf_cap = 0;
    MfBuffers w{};
    uint8_t *inpad = nullptr, *d_scr = nullptr;
    uint64_t *d_offs = nullptr, *d_oofs = nullptr, *d_lens = nullptr, *d_rofs = nullptr, *d_rlens = nullptr;
    uint32_t *d_order = nullptr, *d_seg = nullptr;
    int32_t* d_status = nullptr;
    unsigned* d_next = nullptr;
    uint16_t* d_recs = nullptr;
    // the sliced encode (lzma_enc_session_*): the parse stops / resumes at block boundaries
    uint8_t* slice_state = nullptr;
    uint32_t slice_stop = 0, slice_resume = 0;
    uint64_t pool_cap(uint64_t spk) const {   // one slot per position at most
        uint64_t slots = std::min<uint64_t>(total, (total * spk + 1023) / 1024) + 64;
        return slots * stride;
    }
};

static void pass_plan(Ctx* ctx, EncPass& P, const Derived& d, const uint8_t* d_in, const uint64_t* h_offs, int s0, int s1,
                      uint8_t* d_out, const uint64_t* h_out_offs, bool split) {
    P.d = d;
    P.d_in = d_in;
    P.d_out = d_out;
    P.split = split;
    P.ns = s1 - s0;
    const int ns = P.ns;
    P.in0 = h_offs[s0];
    P.total = h_offs[s1] - P.in0;
    P.offs.assign(ns + 1, 0);
    P.oofs.assign(ns + 1, 0);
    for (int i = 0; i <= ns; i++) { P.offs[i] = h_offs[s0 + i] - P.in0; P.oofs[i] = h_out_offs[s0 + i]; }
    P.wide = false;
    for (int i = 0; i < ns; i++)
        if (P.offs[i + 1] - P.offs[i] >= PairPack<uint32_t>::kMaxStream) P.wide = true;
    P.psz = P.wide ? 8 : 4;
    // longest streams first (work queue order)
    P.order.resize(ns);
    std::iota(P.order.begin(), P.order.end(), 0u);
    std::stable_sort(P.order.begin(), P.order.end(), [&](uint32_t a, uint32_t b) {
        return (P.offs[a + 1] - P.offs[a]) > (P.offs[b + 1] - P.offs[b]);
    });
    P.grid = enc_grid(d, ns);
    P.scr = (enc_scratch_per_block(d) + 255) & ~(size_t)255;
    // overflow pool in slots of ovf_stride(fb) pairs, one slot per position with more
    // than kInlinePairs pairs: start at 1 slot per 16 positions (a retry grows it 4x and
    // remembers the rate for later passes of this context), never more than one per position
    P.stride = ovf_stride(d.fb);
    P.slots_per_k = std::max<uint64_t>(64, ctx->ovf_hint);
    P.ovf_cap = P.pool_cap(P.slots_per_k);
    // coder records (rc.hip) per stream: capacity layout in records, 64-record aligned
    P.rofs.assign(ns + 1, 0);
    for (int i = 0; i < ns; i++) P.rofs[i + 1] = P.rofs[i] + rc_record_bound(P.offs[i + 1] - P.offs[i]);
}

// The layout for the pass's current overflow pool. The pass's live buffers (input copy,
// pass arrays, match lists, overflow pool, the parser's spill scratch: staging to parse)
// come from live[P.slot]; the match finder's scratch from the shared arena. The sync
// form keeps the coder records in the memory of the match finder's buffers (dead after
// the walk); the split form keeps them, and the coder's own arrays, in separate
// allocations (Ctx::split_*) that the next pass's match finder never touches.
static int pass_carve(Ctx* ctx, EncPass& P) {
    const uint64_t T = P.total;
    const int ns = P.ns;
    auto phase1 = [&](Carver& c, MfBuffers& w) {   // buffers only the match finder uses
        // positions need no array of their own (the sorts' first pass takes the index), nor do
        // the chains' own indices; the long-chain lists live in k4's memory after the hash4 sort
        w.k4 = c.take<uint64_t>(T); w.k3 = c.take<uint32_t>(T); w.k2 = c.take<uint32_t>(T); w.ks = c.take<uint64_t>(T);
        w.vs = c.take<uint32_t>(T);
        w.prev3 = c.take<uint32_t>(T);
        w.chain_start = c.take<uint32_t>(T); w.chain_len = c.take<uint32_t>(T);
        w.chain_order = c.take<uint32_t>(T);
        w.cls = c.take<uint32_t>(96);
        w.son = c.take<uint64_t>(4 * T);   // mf.hip WNode: 32 bytes per position
        w.hist = c.take<uint32_t>(sort_hist_words(T, ns));
        w.seg_end = c.take<uint64_t>((size_t)ns + 1);
        w.chain_offs = c.take<uint64_t>((size_t)ns + 1);
    };
    size_t p1_bytes;
    {
        MfBuffers pw{};
        Carver probe(nullptr);
        phase1(probe, pw);
        p1_bytes = probe.off;
    }
    const size_t rec_bytes_all = P.rofs[ns] * 2;
    const size_t union_bytes = P.split ? p1_bytes : std::max<size_t>(p1_bytes, rec_bytes_all);
    auto need_live = [&](Carver& c, EncPass& Q) {
        Q.inpad = c.take<uint8_t>(T + 512);
        Q.d_offs = c.take<uint64_t>(ns + 1);
        Q.d_oofs = c.take<uint64_t>(ns + 1);
        Q.d_order = c.take<uint32_t>(ns);
        Q.d_lens = c.take<uint64_t>(ns);
        Q.d_status = c.take<int32_t>(ns);
        Q.d_next = c.take<unsigned>(4);
        Q.d_rofs = c.take<uint64_t>(ns + 1);
        Q.d_rlens = c.take<uint64_t>(ns);
        Q.d_seg = c.take<uint32_t>((size_t)ns * kRcSegs * kRcSegWords);
        Q.w.pairs = (v4u32*)c.take<uint8_t>(T * rec_bytes(Q.wide));
        Q.w.ovf_off = c.take<uint32_t>(T);
        Q.w.ovf = c.take<uint8_t>(Q.ovf_cap * Q.psz);
        Q.w.ovf_cap = Q.ovf_cap;
        Q.w.ovf_used = c.take<unsigned long long>(1);
        Q.w.err = c.take<int>(1);
        // the parser's spill scratch: the pass's own (in the split form the newer pass's
        // walk runs beside this pass's parse, over the shared match-finder scratch)
        Q.d_scr = c.take<uint8_t>((size_t)Q.grid * Q.scr);
    };
    auto need_shared = [&](Carver& c, EncPass& Q) {   // one pass's keys, sorts, chains and tree at a time
        uint8_t* u = c.take<uint8_t>(union_bytes);
        Q.d_recs = (uint16_t*)u;
        Carver c1(u);
        phase1(c1, Q.w);
    };
    {
        Carver pl(nullptr), ps(nullptr);
        EncPass Q;
        Q.wide = P.wide; Q.ovf_cap = P.ovf_cap; Q.psz = P.psz; Q.grid = P.grid; Q.scr = P.scr;
        need_live(pl, Q);
        need_shared(ps, Q);
        DevBuf& L = ctx->live[P.slot];
        if (pl.off + 4096 > L.n || ps.off + 4096 > ctx->arena_size) {
            // a reallocation waits for everything that may still read the old buffers: the
            // other staged pass's walk, the older pass's parse, the coder's caller
            if (ctx->split_state || ctx->rc_pending) HIPCHK(ctx->device_sync());
            if (!L.ensure(pl.off + 4096)) return ctx->fail(LZMA_E_NOMEM, "device workspace %zu bytes", pl.off);
            if (!ctx->ensure_arena(ps.off + 4096)) return ctx->fail(LZMA_E_NOMEM, "device workspace %zu bytes", ps.off);
        }
    }
    Carver cl(ctx->live[P.slot].as<uint8_t>()), cs(ctx->arena);
    need_live(cl, P);
    need_shared(cs, P);
    P.carved_arena = ctx->arena;
    return LZMA_OK;   // the split form binds its coder records when its parse is enqueued (coder_bind)
}

// The split form: a pass's pointers into the context's shared arena (the match finder's
// scratch) as of now. Another pass's staging
// may have grown, and so moved, them since this pass was carved (it waited for every user
// of the old ones first); the live buffers are the pass's own slot's and do not move.
static int pass_refresh_shared(Ctx* ctx, EncPass& P) {
    if (P.carved_arena == ctx->arena) return LZMA_OK;
    return pass_carve(ctx, P);   // sizes unchanged: no reallocation, the live slot's layout is the same
}

// host arrays through pinned staging (see HostBuf): the pass's later host round trip
// (the match finder's chain count) comes after these copies, so the staging is free
// again when the next pass fills it
static int pass_stage(Ctx* ctx, EncPass& P, hipStream_t st) {
    const size_t pn = (size_t)P.ns + 1;
    if (!ctx->pin.ensure(pn * 8 * 5 + pn * 4 * 2)) return ctx->fail(LZMA_E_NOMEM, "pinned staging");
    uint64_t* p_offs = ctx->pin.as<uint64_t>();
    uint64_t* p_oofs = p_offs + pn;
    uint64_t* p_rofs = p_oofs + pn;
    uint32_t* p_order = (uint32_t*)(p_rofs + pn + pn);
    memcpy(p_offs, P.offs.data(), pn * 8);
    memcpy(p_oofs, P.oofs.data(), pn * 8);
    memcpy(p_rofs, P.rofs.data(), pn * 8);
    memcpy(p_order, P.order.data(), (size_t)P.ns * 4);
    TimedLaunch tl(ctx, "enc_stage", st);
    HIPCHK(hipMemcpyAsync(P.inpad, P.d_in + P.in0, P.total, hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemsetAsync(P.inpad + P.total, 0, 512, st));
    HIPCHK(hipMemcpyAsync(P.d_offs, p_offs, pn * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(P.d_oofs, p_oofs, pn * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(P.d_order, p_order, P.ns * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(P.d_rofs, p_rofs, pn * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(P.d_next, 0, 16, st));
    return LZMA_OK;
}

// the walk on st now (its chain count read back through P's pinned slot), then its verdict
static int walk_now(Ctx* ctx, EncPass& P, hipStream_t st) {
    int rc;
    if ((rc = mf_count_enqueue(ctx, P.w, P.ns, st, P.slot)) ||
        (rc = mf_walk_launch(ctx, P.d, P.inpad, P.d_offs, P.ns, P.total, P.wide, P.w, st, P.slot)))
        return rc;
    HIPCHK(hipStreamSynchronize(st));
    return mf_walk_result(ctx, P.slot);
}

// the walk (or, split form, the verdict of the walk already enqueued: walk_state 1); on a
// full overflow pool, grow it (4x, remembered by the context) and run the pass's match
// finder again from the staging. Returns LZMA_OK or an error; *redone: the match finder
// ran again (its scratch now holds this pass's buffers).
static int pass_mf_back(Ctx* ctx, EncPass& P, hipStream_t st, bool* redone = nullptr) {
    for (int attempt = 0; attempt < 6; attempt++) {
        int rc;
        if (P.walk_state == 1) {
            P.walk_state = 0;
            HIPCHK(hipEventSynchronize(ctx->walk_done[P.slot]));
            rc = mf_walk_result(ctx, P.slot);
        } else rc = walk_now(ctx, P, st);
        if (rc != LZMA_E_OVERFLOW) return rc;
        if (P.slots_per_k >= 1024) return ctx->fail(LZMA_E_INTERNAL, "overflow pool full at one slot per position");
        P.slots_per_k = std::min<uint64_t>(1024, P.slots_per_k * 4);
        ctx->ovf_hint = P.slots_per_k;
        P.ovf_cap = P.pool_cap(P.slots_per_k);
        if (redone) *redone = true;
        HIPCHK(ctx->device_sync());   // rare: the staging below reuses pinned memory other copies may read
        if ((rc = pass_carve(ctx, P)) || (rc = pass_stage(ctx, P, st)) ||
            (rc = mf_front(ctx, P.d, P.inpad, P.d_offs, P.ns, P.total, P.wide, P.w, st)))
            return rc;
    }
    return ctx->fail(LZMA_E_NOMEM, "match-pair overflow pool kept overflowing");
}

static int pass_parse(Ctx* ctx, EncPass& P, hipStream_t st) {
    // the walk-subset timing hook leaves the skipped positions' records holding the walk's
    // inputs (mf_prev2_kernel), not match lists: such a pass is never parsed
    if (exp_env("LZG_WALK_ONLY")) return ctx->fail(LZMA_E_PARAM, "LZG_WALK_ONLY (a walk timing experiment): no parse");
    EncArgs a{};
    a.in = P.inpad; a.offs = P.d_offs; a.order = P.d_order; a.nstreams = P.ns; a.next = P.d_next;
    a.pairs = P.w.pairs; a.ovf_off = P.w.ovf_off; a.ovf = P.w.ovf;
    a.recs = P.d_recs; a.rec_offs = P.d_rofs; a.rec_lens = P.d_rlens; a.out_lens = P.d_lens; a.status = P.d_status;
    a.scratch = P.d_scr; a.scratch_stride = P.scr;
    a.lit_stride = (enc_lit_bytes(P.d) + 255) & ~(size_t)255;
    if (!ctx->ensure_litbuf((size_t)P.grid * a.lit_stride + 256)) return ctx->fail(LZMA_E_NOMEM, "literal-coder tables");
    a.lit_scratch = ctx->litbuf;
    const Derived& d = P.d;
    a.fb = d.fb; a.lc = d.lc; a.lp = d.lp; a.pb = d.pb; a.eos = d.eos;
    a.dist_table_size = d.dist_table_size; a.len_table_size = d.len_table_size;
    a.lit_in_lds = enc_lit_in_lds(d, P.grid);
    a.pair_bytes = P.wide ? 8 : 4;
    LZG_TRACE(ctx, st, "encode pass: %d streams, %llu bytes, grid %d", P.ns, (unsigned long long)P.total, P.grid);
    DebugWatch watch;
    if (ctx->debug) { watch.start(16); a.dbg = watch.dev; }
#ifdef LZG_PROF
    uint64_t* d_prof = nullptr;
    HIPCHK(hipMalloc(&d_prof, (size_t)P.ns * kProfSlots * 8));
    HIPCHK(hipMemsetAsync(d_prof, 0, (size_t)P.ns * kProfSlots * 8, st));
    a.prof = d_prof;
#endif
    // a pipelined caller's decoder (another context) may still hold CUs: the
    // parser needs every stream resident from its start, so it waits for it. The
    // fence is read under the live-context lock: lzma_ctx_destroy on another thread
    // clears it (and destroys the event) only under that lock.
    if (ctx->fence) {
        std::lock_guard<std::mutex> g(g_ctx_lock);
        const Ctx* f = ctx->fence;
        if (f && g_live_ctx.count(const_cast<Ctx*>(f)) && f->dec_pending) HIPCHK(hipStreamWaitEvent(st, f->dec_done, 0));
    }
    if (P.split) {   // a staged pass's walk waits for this point (runtime.hip enc_parse_dev_async)
        if (!ctx->parse_start && hipEventCreateWithFlags(&ctx->parse_start, hipEventDisableTiming) != hipSuccess)
            return ctx->fail(LZMA_E_DEVICE, "parse event");
        HIPCHK(hipEventRecord(ctx->parse_start, st));
    }
    int rc;
    if (P.slice_state) {
        a.slice_state = P.slice_state;
        a.slice_stride = 0;   // one stream
        a.slice_stop = P.slice_stop;
        a.slice_resume = P.slice_resume;
        rc = launch_encoder_sliced(ctx, a, P.wide, P.grid, st);
    } else {
        rc = launch_encoder(ctx, a, P.wide, P.grid, st);
    }
    if (rc) return rc;
    LZG_TRACE(ctx, st, "enc_parse done");
    watch.stop();
#ifdef LZG_PROF
    report_profile(d_prof, P.ns, P.total, st);
    hipFree(d_prof);
#endif
    return LZMA_OK;
}

// the range coder over the parser's records (the coder's arrays: the pass's own, or the
// split form's copies)
static int pass_rc(Ctx* ctx, EncPass& P, uint64_t* rofs, uint64_t* rlens, uint32_t* order, int32_t* status, uint64_t* oofs,
                   uint64_t* lens, uint32_t* seg, hipStream_t st, const RcArgs* slice = nullptr) {
    RcArgs ra{};
    if (slice) ra = *slice;   // the sliced encode's coder state and flush (sliced, flush, init_state, end_state)
    else ra.flush = 1;
    ra.recs = P.d_recs; ra.rec_offs = rofs; ra.rec_lens = rlens; ra.order = order; ra.nstreams = P.ns;
    ra.status = status; ra.out = P.d_out; ra.out_offs = oofs; ra.out_lens = lens; ra.seg = seg;
    int rc = launch_rc(ctx, ra, st);
    LZG_TRACE(ctx, st, "enc_rc done");
    return rc;
}

// one synchronous pass (dump != null: stop after the match finder and copy its output
// to the host)
static int encode_pass(Ctx* ctx, const Derived& d, const uint8_t* d_in, const uint64_t* h_offs, int s0, int s1,
                       uint8_t* d_out, const uint64_t* h_out_offs, uint64_t* h_out_lens, int32_t* h_status,
                       hipStream_t st, MatchDump* dump = nullptr) {
    if (ctx->dec_pending) return ctx->fail(LZMA_E_PARAM, "an asynchronous decode is in flight: lzma_dec_batch_dev_wait first");
    if (ctx->split_state || ctx->rc_pending)
        return ctx->fail(LZMA_E_PARAM, "a split encode is in flight on this context: lzma_enc_parse_dev_async / _wait first");
    if (ctx->session) return ctx->fail(LZMA_E_PARAM, "an encode session is open on this context: lzma_enc_session_end first");
    EncPass P;
    pass_plan(ctx, P, d, d_in, h_offs, s0, s1, d_out, h_out_offs, false);
    // Nothing is staged, so either live slot is free: take the larger one. A split schedule
    // that stages one batch at a time (the fenced bench) only ever grows slot 1, and a
    // synchronous pass fixed to slot 0 then paid a first hipMalloc of ~46 B per input byte
    // (bench.py's `sequential` leg after the pipelined loop: 1,441.6 ms in the driver's
    // round-5 record; tests/test_async_emulated.py counts the allocations).
    P.slot = ctx->live[1].n > ctx->live[0].n ? 1 : 0;
    int rc;
    if ((rc = pass_carve(ctx, P)) || (rc = pass_stage(ctx, P, st)) ||
        (rc = mf_front(ctx, P.d, P.inpad, P.d_offs, P.ns, P.total, P.wide, P.w, st)) || (rc = pass_mf_back(ctx, P, st)))
        return rc;
    const int ns = P.ns;
    const size_t pn = (size_t)ns + 1;
    uint64_t* p_lens = ctx->pin.as<uint64_t>() + 3 * pn;
    int32_t* p_status = (int32_t*)((uint32_t*)(p_lens + pn) + pn);
    if (dump) {
        const uint64_t total = P.total;
        dump->wide = P.wide;
        dump->stride = (uint32_t)P.stride;
        dump->ovf_off.resize(total);
        dump->recs.resize(total * rec_bytes(P.wide));
        HIPCHK(hipMemcpyAsync(p_lens, P.w.ovf_used, 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        const unsigned long long used = p_lens[0];
        dump->ovf.resize(std::min<uint64_t>(used * P.stride, P.ovf_cap) * P.psz);
        if (total) {
            HIPCHK(hipMemcpyAsync(dump->ovf_off.data(), P.w.ovf_off, total * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(dump->recs.data(), P.w.pairs, dump->recs.size(), hipMemcpyDeviceToHost, st));
        }
        if (!dump->ovf.empty()) HIPCHK(hipMemcpyAsync(dump->ovf.data(), P.w.ovf, dump->ovf.size(), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        return LZMA_OK;
    }
    if ((rc = pass_parse(ctx, P, st)) ||
        (rc = pass_rc(ctx, P, P.d_rofs, P.d_rlens, P.d_order, P.d_status, P.d_oofs, P.d_lens, P.d_seg, st)))
        return rc;
    HIPCHK(hipMemcpyAsync(p_lens, P.d_lens, ns * 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(p_status, P.d_status, ns * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    memcpy(h_out_lens + s0, p_lens, (size_t)ns * 8);
    memcpy(h_status + s0, p_status, (size_t)ns * 4);
    return LZMA_OK;
}

static int check_batch(Ctx* ctx, const uint64_t* h_offs, const uint64_t* h_out_offs, int nstreams) {
    for (int i = 0; i < nstreams; i++) {
        if (h_offs[i + 1] < h_offs[i] || h_out_offs[i + 1] < h_out_offs[i]) return ctx->fail(LZMA_E_PARAM, "offsets not monotone");
        if (h_offs[i + 1] - h_offs[i] >= (1ull << 31)) return ctx->fail(LZMA_E_PARAM, "stream %d >= 2 GiB", i);
    }
    return LZMA_OK;
}

static int encode_batch_dev(Ctx* ctx, const lzma_params* p, const uint8_t* d_in, const uint64_t* h_offs, int nstreams,
                            uint8_t* d_out, const uint64_t* h_out_offs, uint64_t* h_out_lens, hipStream_t st) {
    Derived d;
    if (derive(*p, d) != LZMA_OK) return ctx->fail(LZMA_E_PARAM, "invalid lzma_params");
    if (nstreams < 0) return ctx->fail(LZMA_E_PARAM, "nstreams < 0");
    if (nstreams == 0) return LZMA_OK;
    int crc = check_batch(ctx, h_offs, h_out_offs, nstreams);
    if (crc) return crc;
    std::vector<int32_t> status(nstreams, 0);
    int s0 = 0;
    // h_out_lens doubles as a diagnostic for LZMA_E_INTERNAL: (reason << 32) | position
    while (s0 < nstreams) {
        int s1 = s0 + 1;
        // bytes bound the match-finder workspace; the stream count bounds the
        // per-workgroup parser scratch (one workgroup per stream)
        // the radix sorts and stream selection take an int item count: a pass stays below 2^31 bytes
        const uint64_t pass_cap = std::min<uint64_t>(ctx->batch_bytes, (1ull << 31) - 1);
        while (s1 < nstreams && s1 - s0 < kMaxStreamsPerPass && h_offs[s1 + 1] - h_offs[s0] <= pass_cap) s1++;
        int rc = encode_pass(ctx, d, d_in, h_offs, s0, s1, d_out, h_out_offs, h_out_lens, status.data(), st);
        if (rc) return rc;
        s0 = s1;
    }
    for (int i = 0; i < nstreams; i++)
        if (status[i] != LZMA_OK)
            return ctx->fail(status[i], status[i] == LZMA_E_OVERFLOW ? "stream %d: output capacity too small%.0llu"
                                                                     : "stream %d: encoder consistency check tripped (%llx)",
                             i, (unsigned long long)h_out_lens[i]);
    return LZMA_OK;
}

// ---- the split encode (lzma_enc_stage_dev / lzma_enc_parse_dev_async / _wait)
// The coder's per-stream arrays, copied out of the pass arrays in one launch once the
// parser is done: the next pass's staging rewrites the pass arrays while the coder runs.
struct CoderArrays {
    uint64_t *rofs, *rlens, *oofs, *lens;
    uint32_t *order, *seg;
    int32_t* status;
};
static CoderArrays coder_arrays(Ctx* ctx, int slot, int ns) {
    Carver c(ctx->split_coder[slot].as<uint8_t>());
    CoderArrays r;
    r.rofs = c.take<uint64_t>(ns + 1); r.oofs = c.take<uint64_t>(ns + 1);
    r.rlens = c.take<uint64_t>(ns); r.lens = c.take<uint64_t>(ns);
    r.order = c.take<uint32_t>(ns); r.status = c.take<int32_t>(ns);
    r.seg = c.take<uint32_t>((size_t)ns * kRcSegs * kRcSegWords);
    return r;
}
__global__ void coder_arrays_kernel(int ns, const uint64_t* rofs, const uint64_t* rlens, const uint64_t* oofs, const uint64_t* lens,
                                    const uint32_t* order, const int32_t* status, CoderArrays o) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i <= ns; i += gridDim.x * blockDim.x) {
        o.rofs[i] = rofs[i];
        o.oofs[i] = oofs[i];
        if (i < ns) { o.rlens[i] = rlens[i]; o.lens[i] = lens[i]; o.order[i] = order[i]; o.status[i] = status[i]; }
    }
}

// The split form holds up to two staged passes (slots 0 / 1 of the live buffers, pinned
// words and events) and up to two range coders in flight (coder_bind). Without a parse
// fence bench.py keeps two batches staged: batch k + 1's keys and sorts (which need LDS)
// run on st before batch k's parser, its walk (no LDS, latency-bound) on the walk stream
// beside that parser, and batch k + 2's staging waits for that walk, as its match finder
// reuses the same scratch. With a fence it stages one batch at a time (stage k + 1 after
// parse_async k).
// The split form's coder buffers (records, the coder's per-stream arrays, the pinned
// lengths and verdicts): two sets, one per coder in flight. A pass takes set 0 unless the
// coder in flight holds it; so a caller that collects each coder before the next parse
// allocates one set. Returns the set.
static int coder_bind(Ctx* ctx, EncPass& P, int* set) {
    const int rb = (ctx->rc_pending == 1 && ctx->rc_slot[0] == 0) ? 1 : 0;   // no coder in flight holds rb
    const int ns = P.ns;
    const size_t rec_bytes_all = P.rofs[ns] * 2;
    const size_t coder_bytes = (size_t)(ns + 1) * 8 * 4 + (size_t)ns * 8 + (size_t)ns * kRcSegs * kRcSegWords * 4 + 4096;
    if (!ctx->split_recs[rb].ensure(std::max<size_t>(rec_bytes_all, 256)) || !ctx->split_coder[rb].ensure(coder_bytes) ||
        !ctx->pin_rc[rb].ensure((size_t)ns * 12 + 16))
        return ctx->fail(LZMA_E_NOMEM, "coder records %zu bytes", rec_bytes_all);
    P.d_recs = ctx->split_recs[rb].as<uint16_t>();
    *set = rb;
    return LZMA_OK;
}

// the coder's per-stream lengths and verdicts into pinned host memory, on the coder stream
// behind the coder (a kernel, not a copy: a device-to-host copy queued behind the coder
// would hold a copy engine that other streams' copies need)
__global__ void coder_out_kernel(int ns, const uint64_t* lens, const int32_t* status, uint64_t* h_lens, int32_t* h_status) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < ns; i += gridDim.x * blockDim.x) {
        h_lens[i] = lens[i];
        h_status[i] = status[i];
    }
}

static int enc_stage_dev(Ctx* ctx, const lzma_params* p, const uint8_t* d_in, const uint64_t* h_offs, int nstreams,
                         uint8_t* d_out, const uint64_t* h_out_offs, hipStream_t st) {
    if (ctx->dec_pending) return ctx->fail(LZMA_E_PARAM, "an asynchronous decode is in flight: lzma_dec_batch_dev_wait first");
    if (ctx->split_state >= 2) return ctx->fail(LZMA_E_PARAM, "two batches are already staged: lzma_enc_parse_dev_async first");
    if (ctx->session) return ctx->fail(LZMA_E_PARAM, "an encode session is open on this context: lzma_enc_session_end first");
    Derived d;
    if (derive(*p, d) != LZMA_OK) return ctx->fail(LZMA_E_PARAM, "invalid lzma_params");
    if (nstreams <= 0) return ctx->fail(LZMA_E_PARAM, "the split form needs at least one stream");
    int rc = check_batch(ctx, h_offs, h_out_offs, nstreams);
    if (rc) return rc;
    const uint64_t pass_cap = std::min<uint64_t>(ctx->batch_bytes, (1ull << 31) - 1);
    if (nstreams > kMaxStreamsPerPass || (nstreams > 1 && h_offs[nstreams] - h_offs[0] > pass_cap))
        return ctx->fail(LZMA_E_PARAM, "the split form takes one pass: at most %d streams and batch_bytes of input", kMaxStreamsPerPass);
    // Alone, the batch takes the slot the last consumed batch had (its parse, still running,
    // comes first on st, and a reallocation waits for it): a caller that never stages two
    // batches uses one live slot. The second staged batch takes the other slot.
    if (ctx->split_state == 0) ctx->split_head = (ctx->split_head + 1) % 2;
    const int slot = (ctx->split_head + ctx->split_state) % 2;
    for (int k = 0; k < 2; k++) {
        if (!ctx->walk_done[k] && hipEventCreateWithFlags(&ctx->walk_done[k], hipEventDisableTiming) != hipSuccess)
            return ctx->fail(LZMA_E_DEVICE, "walk event");
    }
    if (ctx->split_state == 1) {
        // the older staged pass's walk reads the match-finder scratch this staging rewrites
        EncPass& O = *ctx->split_pass[ctx->split_head];
        if (O.walk_state == 0) {
            if ((rc = mf_walk_launch(ctx, O.d, O.inpad, O.d_offs, O.ns, O.total, O.wide, O.w, st, O.slot))) return rc;
            HIPCHK(hipEventRecord(ctx->walk_done[O.slot], st));
            O.walk_state = 1;
        } else HIPCHK(hipStreamWaitEvent(st, ctx->walk_done[O.slot], 0));
    }
    if (!ctx->split_pass[slot]) ctx->split_pass[slot] = new (std::nothrow) EncPass;
    if (!ctx->split_pass[slot]) return ctx->fail(LZMA_E_NOMEM, "split pass");
    EncPass& P = *ctx->split_pass[slot];
    P = EncPass();
    pass_plan(ctx, P, d, d_in, h_offs, 0, nstreams, d_out, h_out_offs, true);
    P.slot = slot;
    if ((rc = pass_carve(ctx, P)) || (rc = pass_stage(ctx, P, st)) ||
        (rc = mf_front(ctx, P.d, P.inpad, P.d_offs, P.ns, P.total, P.wide, P.w, st)) ||
        (rc = mf_count_enqueue(ctx, P.w, P.ns, st, slot)))
        return rc;
    // Alone (nothing older staged) and without a parse fence, the walk too: it then runs as
    // soon as the sorts are done instead of when the caller next enqueues a parse. Its grid
    // is sized by a host read of the chain count, so this call then waits for the work ahead
    // of it on st. With a fence, the caller's decode is on the critical path and must not
    // wait behind that: the walk stays in lzma_enc_parse_dev_async.
    bool fenced;
    {
        std::lock_guard<std::mutex> g(g_ctx_lock);
        fenced = ctx->fence != nullptr;
    }
    if (ctx->split_state == 0 && !fenced) {
        if ((rc = mf_walk_launch(ctx, P.d, P.inpad, P.d_offs, P.ns, P.total, P.wide, P.w, st, slot))) return rc;
        HIPCHK(hipEventRecord(ctx->walk_done[slot], st));
        P.walk_state = 1;
    }
    ctx->split_state++;
    return LZMA_OK;
}

// Experiment build only: fail the named step of lzma_enc_parse_dev_async (LZG_FAIL_AT =
// "walk2": the newer staged batch's walk launch; "rc": the coder launch), so the CPU
// emulation can check that a failure after the oldest batch is consumed drops every staged
// batch (tests/test_async_emulated.py).
static bool inject_fail(const char* step) {
    const char* e = exp_env("LZG_FAIL_AT");
    return e && strcmp(e, step) == 0;
}

static int enc_parse_dev_async_body(Ctx* ctx, hipStream_t st);

// A refusal (LZMA_E_PARAM before anything is consumed) leaves the staged batches as they were.
// Once the oldest staged batch is consumed, any failure drops every staged batch (split_state
// 0, the newer batch's walk forgotten) and is never reported as LZMA_E_PARAM, so a caller
// (lzma_amd's wrapper) can tell the two apart by the code alone (include/lzma_mi355x.h).
static int enc_parse_dev_async(Ctx* ctx, hipStream_t st) {
    if (!ctx->split_state) return ctx->fail(LZMA_E_PARAM, "nothing staged: lzma_enc_stage_dev first");
    if (ctx->rc_pending >= 2) return ctx->fail(LZMA_E_PARAM, "two coders are in flight: lzma_enc_parse_dev_wait first");
    const int rc = enc_parse_dev_async_body(ctx, st);
    if (rc == LZMA_OK) return rc;
    ctx->split_state = 0;
    for (int k = 0; k < 2; k++)
        if (ctx->split_pass[k]) ctx->split_pass[k]->walk_state = 0;
    // what was enqueued before the failure (the newer batch's walk, this batch's parser) may
    // still run over the buffers the next staging reuses: let it drain (a failure path only)
    (void)ctx->device_sync();
    return rc == LZMA_E_PARAM ? LZMA_E_INTERNAL : rc;
}

static int enc_parse_dev_async_body(Ctx* ctx, hipStream_t st) {
    EncPass& P = *ctx->split_pass[ctx->split_head];
    // from here on the oldest staged pass is consumed (or failed)
    ctx->split_head = (ctx->split_head + 1) % 2;
    ctx->split_state--;
    EncPass* Q = ctx->split_state ? ctx->split_pass[ctx->split_head] : nullptr;   // the newer staged pass
    int rc;
    bool redone = false;
    if ((rc = pass_mf_back(ctx, P, st, &redone))) return rc;
    if (redone && Q) {   // P's match finder ran again over the scratch Q's staging had filled
        if ((rc = pass_refresh_shared(ctx, *Q)) || (rc = pass_stage(ctx, *Q, st)) || (rc = mf_front(ctx, Q->d, Q->inpad, Q->d_offs, Q->ns, Q->total, Q->wide, Q->w, st)) ||
            (rc = mf_count_enqueue(ctx, Q->w, Q->ns, st, Q->slot)))
            return rc;
        Q->walk_state = 0;
    }
    if (exp_env("LZG_PROBE_WALK_ONLY")) return LZMA_OK;   // experiment build: concurrency probe (tools/overlap_probe.py)
    int ps;   // the coder set
    if ((rc = pass_refresh_shared(ctx, P)) || (rc = coder_bind(ctx, P, &ps)) || (rc = pass_parse(ctx, P, st))) return rc;
    if (!ctx->rc_stream && hipStreamCreateWithFlags(&ctx->rc_stream, hipStreamNonBlocking) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "coder stream");
    // The newer staged pass's walk beside this parse, on the walk stream: launched after the
    // parser (its waves are resident first; the walk's take the rest), once its sorts are
    // done (its chain count sizes the grid), and before the coder is enqueued: HIP streams
    // share hardware queues (GPU_MAX_HW_QUEUES), and a walk queued behind the coder (which
    // waits for this parse) would run after it, with the caller's copies behind the walk.
    if (Q && Q->walk_state == 0) {
        if (!ctx->walk_stream && hipStreamCreateWithFlags(&ctx->walk_stream, hipStreamNonBlocking) != hipSuccess)
            return ctx->fail(LZMA_E_DEVICE, "walk stream");
        // not before this parse starts (with a fence it waits for the previous decode): the
        // walk then runs beside this parse, and does not take the CUs the parse is waiting for
        HIPCHK(hipStreamWaitEvent(ctx->walk_stream, ctx->parse_start, 0));
        if (inject_fail("walk2")) return ctx->fail(LZMA_E_DEVICE, "injected failure (LZG_FAIL_AT=walk2)");
        if ((rc = mf_walk_launch(ctx, Q->d, Q->inpad, Q->d_offs, Q->ns, Q->total, Q->wide, Q->w, ctx->walk_stream, Q->slot)))
            return rc;
        HIPCHK(hipEventRecord(ctx->walk_done[Q->slot], ctx->walk_stream));
        Q->walk_state = 1;
    }
    if (!ctx->parse_done[ps] && hipEventCreateWithFlags(&ctx->parse_done[ps], hipEventDisableTiming) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "parse event");
    if (!ctx->rc_done[ps] && hipEventCreateWithFlags(&ctx->rc_done[ps], hipEventDisableTiming) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "coder event");
    // The copy of the pass arrays runs on the caller's stream, ahead of parse_done: a
    // later lzma_enc_stage_dev on that stream rewrites the pass arrays (a new batch's
    // offsets, order, status), and stream order keeps that behind this copy. Only the
    // coder itself runs on the coder stream.
    const CoderArrays ca = coder_arrays(ctx, ps, P.ns);
    hipLaunchKernelGGL(coder_arrays_kernel, dim3((P.ns + 256) / 256), dim3(256), 0, st, P.ns, P.d_rofs, P.d_rlens,
                       P.d_oofs, P.d_lens, P.d_order, P.d_status, ca);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->parse_done[ps], st));
    HIPCHK(hipStreamWaitEvent(ctx->rc_stream, ctx->parse_done[ps], 0));
    if (inject_fail("rc")) return ctx->fail(LZMA_E_DEVICE, "injected failure (LZG_FAIL_AT=rc)");
    if ((rc = pass_rc(ctx, P, ca.rofs, ca.rlens, ca.order, ca.status, ca.oofs, ca.lens, ca.seg, ctx->rc_stream))) return rc;
    uint64_t* h_lens = ctx->pin_rc[ps].as<uint64_t>();
    hipLaunchKernelGGL(coder_out_kernel, dim3((P.ns + 255) / 256), dim3(256), 0, ctx->rc_stream, P.ns, ca.lens, ca.status,
                       h_lens, (int32_t*)(h_lens + P.ns));
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ctx->rc_done[ps], ctx->rc_stream));
    ctx->rc_slot[ctx->rc_pending] = ps;
    ctx->rc_ns[ctx->rc_pending] = P.ns;
    ctx->rc_pending++;
    return LZMA_OK;
}

static int enc_parse_dev_wait(Ctx* ctx, uint64_t* h_out_lens) {
    if (!ctx->rc_pending) return ctx->fail(LZMA_E_PARAM, "no coder in flight: lzma_enc_parse_dev_async first");
    const int slot = ctx->rc_slot[0], ns = ctx->rc_ns[0];   // the oldest coder
    ctx->rc_slot[0] = ctx->rc_slot[1];
    ctx->rc_ns[0] = ctx->rc_ns[1];
    ctx->rc_pending--;
    HIPCHK(hipEventSynchronize(ctx->rc_done[slot]));   // coder_out_kernel has written the pinned words
    const uint64_t* p_lens = ctx->pin_rc[slot].as<uint64_t>();
    const int32_t* p_status = (const int32_t*)(p_lens + ns);
    memcpy(h_out_lens, p_lens, (size_t)ns * 8);
    for (int i = 0; i < ns; i++)
        if (p_status[i] != LZMA_OK)
            return ctx->fail(p_status[i], p_status[i] == LZMA_E_OVERFLOW ? "stream %d: output capacity too small%.0llu"
                                                                         : "stream %d: encoder consistency check tripped (%llx)",
                             i, (unsigned long long)p_lens[i]);
    return LZMA_OK;
}

// Enqueues one batch decode on st. h_* arrays are read before the first copy
// completes only when `pinned` is false (the copies are then staged by the
// runtime); lens/status land in h_out_lens / h_status once st reaches them.
static int decode_enqueue(Ctx* ctx, const uint8_t props[5], const uint8_t* d_in, const uint64_t* h_in_offs, int nstreams,
                          const int64_t* h_out_sizes, uint8_t* d_out, const uint64_t* h_out_offs, uint64_t* h_out_lens,
                          int32_t* h_status, uint32_t* h_order, hipStream_t st) {
    lzma_params p;
    if (lzma_read_props(props, &p) != LZMA_OK) return ctx->fail(LZMA_E_PARAM, "bad properties (Decoder.SetDecoderProperties false)");
    for (int i = 0; i < nstreams; i++) {   // the decoder kernel keeps 32-bit input positions
        if (h_in_offs[i + 1] < h_in_offs[i] || h_in_offs[i + 1] - h_in_offs[i] >= 0xFFFFFFFFull)
            return ctx->fail(LZMA_E_PARAM, "compressed stream %d: bad offsets or >= 4 GiB", i);
        if (h_out_offs[i + 1] < h_out_offs[i] || h_out_offs[i + 1] - h_out_offs[i] >= 0xFFFFFFFFull)
            return ctx->fail(LZMA_E_PARAM, "output region %d: offsets not monotone or >= 4 GiB", i);
    }
    uint32_t dict = (uint32_t)props[1] | ((uint32_t)props[2] << 8) | ((uint32_t)props[3] << 16) | ((uint32_t)props[4] << 24);
    const uint32_t lc = (uint32_t)p.lc, lp = (uint32_t)p.lp, pb = (uint32_t)p.pb;
    const uint32_t lit_lds = 0;   // literal coders always in the per-stream HBM scratch (dec.hip)
    for (int i = 0; i < nstreams; i++) h_order[i] = (uint32_t)i;
    std::stable_sort(h_order, h_order + nstreams, [&](uint32_t a, uint32_t b) {
        return (h_out_offs[a + 1] - h_out_offs[a]) > (h_out_offs[b + 1] - h_out_offs[b]);
    });
    const int grid = dec_grid(lc, lp, lit_lds, nstreams);
    const size_t scr = lit_lds ? 0 : ((dec_scratch_per_block(lc, lp) + 255) & ~(size_t)255);
    Carver probe(nullptr);
    probe.take<uint64_t>(nstreams + 1); probe.take<int64_t>(nstreams); probe.take<uint64_t>(nstreams + 1);
    probe.take<uint64_t>(nstreams); probe.take<int32_t>(nstreams); probe.take<uint32_t>(nstreams);
    probe.take<unsigned>(4);
    if (!ctx->ensure_arena(probe.off + 4096)) return ctx->fail(LZMA_E_NOMEM, "decoder workspace");
    Carver c(ctx->arena);
    uint64_t* d_in_offs = c.take<uint64_t>(nstreams + 1);
    int64_t* d_sizes = c.take<int64_t>(nstreams);
    uint64_t* d_oofs = c.take<uint64_t>(nstreams + 1);
    uint64_t* d_lens = c.take<uint64_t>(nstreams);
    int32_t* d_status = c.take<int32_t>(nstreams);
    uint32_t* d_order = c.take<uint32_t>(nstreams);
    unsigned* d_next = c.take<unsigned>(4);
    if (!ctx->ensure_litbuf((size_t)grid * scr + 16)) return ctx->fail(LZMA_E_NOMEM, "decoder literal-coder tables");
    uint8_t* d_scr = ctx->litbuf;
    HIPCHK(hipMemcpyAsync(d_in_offs, h_in_offs, (nstreams + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_sizes, h_out_sizes, nstreams * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_oofs, h_out_offs, (nstreams + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_order, h_order, nstreams * 4, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(d_next, 0, 16, st));
    DecArgs a{};
    a.in = d_in; a.in_offs = d_in_offs; a.out_sizes = d_sizes; a.out = d_out; a.out_offs = d_oofs;
    a.out_lens = d_lens; a.status = d_status; a.order = d_order; a.nstreams = nstreams; a.next = d_next;
    a.scratch = d_scr; a.scratch_stride = scr; a.lc = lc; a.lp = lp; a.pb = pb;
    a.dict_check = dict > 1 ? dict : 1;
    a.lit_in_lds = lit_lds;
    int rc = launch_decoder(ctx, a, grid, st);
    if (rc) return rc;
    if (h_out_lens) HIPCHK(hipMemcpyAsync(h_out_lens, d_lens, nstreams * 8, hipMemcpyDeviceToHost, st));
    if (h_status) HIPCHK(hipMemcpyAsync(h_status, d_status, nstreams * 4, hipMemcpyDeviceToHost, st));
    return LZMA_OK;
}

static int decode_batch_dev_async(Ctx* ctx, const uint8_t props[5], const uint8_t* d_in, const uint64_t* h_in_offs,
                                  int nstreams, const int64_t* h_out_sizes, uint8_t* d_out, const uint64_t* h_out_offs,
                                  hipStream_t st);
static int decode_batch_dev_wait(Ctx* ctx, uint64_t* h_out_lens, int32_t* h_status);

static int decode_batch_dev(Ctx* ctx, const uint8_t props[5], const uint8_t* d_in, const uint64_t* h_in_offs, int nstreams,
                            const int64_t* h_out_sizes, uint8_t* d_out, const uint64_t* h_out_offs, uint64_t* h_out_lens,
                            int32_t* h_status, hipStream_t st) {
    if (ctx->dec_pending) return ctx->fail(LZMA_E_PARAM, "an asynchronous decode is in flight: lzma_dec_batch_dev_wait first");
    int rc = decode_batch_dev_async(ctx, props, d_in, h_in_offs, nstreams, h_out_sizes, d_out, h_out_offs, st);
    if (rc) return rc;
    return decode_batch_dev_wait(ctx, h_out_lens, h_status);
}

// The asynchronous form: every host array is staged in the context's pinned
// buffer first, so the call returns as soon as the work is enqueued.
static int decode_batch_dev_async(Ctx* ctx, const uint8_t props[5], const uint8_t* d_in, const uint64_t* h_in_offs,
                                  int nstreams, const int64_t* h_out_sizes, uint8_t* d_out, const uint64_t* h_out_offs,
                                  hipStream_t st) {
    if (ctx->dec_pending) return ctx->fail(LZMA_E_PARAM, "an asynchronous decode is already in flight on this context");
    if (ctx->split_state || ctx->rc_pending)   // the decode carves the arena the staged pass holds
        return ctx->fail(LZMA_E_PARAM, "a split encode is in flight on this context: lzma_enc_parse_dev_async / _wait first");
    if (ctx->session) return ctx->fail(LZMA_E_PARAM, "an encode session is open on this context: lzma_enc_session_end first");
    if (nstreams <= 0) return nstreams == 0 ? LZMA_OK : ctx->fail(LZMA_E_PARAM, "nstreams < 0");
    const size_t n = (size_t)nstreams;
    const size_t words = (n + 1) * 3 + n + (n + 1) / 2 * 2 + 2;   // in_offs, sizes, out_offs, lens, order + status
    if (words > ctx->dec_host_words) {
        if (ctx->dec_host) hipHostFree(ctx->dec_host);
        ctx->dec_host = nullptr;
        ctx->dec_host_words = 0;
        ctx->count_alloc(words * 8);
        if (hipHostMalloc((void**)&ctx->dec_host, words * 8, hipHostMallocDefault) != hipSuccess)
            return ctx->fail(LZMA_E_NOMEM, "pinned decode staging");
        ctx->dec_host_words = words;
    }
    if (!ctx->dec_done && hipEventCreateWithFlags(&ctx->dec_done, hipEventDisableTiming) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "decode event");
    uint64_t* in_offs = ctx->dec_host;
    int64_t* sizes = (int64_t*)(in_offs + n + 1);
    uint64_t* out_offs = (uint64_t*)(sizes + n + 1);
    uint64_t* lens = out_offs + n + 1;
    uint32_t* order = (uint32_t*)(lens + n);
    int32_t* status = (int32_t*)(order + (n + 1) / 2 * 2);
    memcpy(in_offs, h_in_offs, (n + 1) * 8);
    memcpy(sizes, h_out_sizes, n * 8);
    memcpy(out_offs, h_out_offs, (n + 1) * 8);
    // no device-to-host copy is queued behind the kernel: a copy waiting on the decode
    // would hold the copy engine, and other streams' copies would queue behind it
    // until the decode ends (_wait copies the results once the kernel is done)
    int rc = decode_enqueue(ctx, props, d_in, in_offs, nstreams, sizes, d_out, out_offs, nullptr, nullptr, order, st);
    if (rc) return rc;
    HIPCHK(hipEventRecord(ctx->dec_done, st));
    ctx->dec_pending = nstreams;
    ctx->dec_stream = st;
    return LZMA_OK;
}

static int decode_batch_dev_wait(Ctx* ctx, uint64_t* h_out_lens, int32_t* h_status) {
    if (!ctx->dec_pending) return LZMA_OK;
    const size_t n = (size_t)ctx->dec_pending;
    ctx->dec_pending = 0;
    HIPCHK(hipEventSynchronize(ctx->dec_done));
    uint64_t* lens = ctx->dec_host + (n + 1) * 3;
    int32_t* status = (int32_t*)((uint32_t*)(lens + n) + (n + 1) / 2 * 2);
    {   // the decoder's outputs sit at the front of the arena (decode_enqueue's carving)
        Carver c(ctx->arena);
        c.take<uint64_t>(n + 1); c.take<int64_t>(n); c.take<uint64_t>(n + 1);
        const uint64_t* d_lens = c.take<uint64_t>(n);
        const int32_t* d_status = c.take<int32_t>(n);
        HIPCHK(hipMemcpyAsync(lens, d_lens, n * 8, hipMemcpyDeviceToHost, ctx->dec_stream));
        HIPCHK(hipMemcpyAsync(status, d_status, n * 4, hipMemcpyDeviceToHost, ctx->dec_stream));
        HIPCHK(hipStreamSynchronize(ctx->dec_stream));
    }
    if (h_out_lens) memcpy(h_out_lens, lens, n * 8);
    if (h_status) memcpy(h_status, status, n * 4);
    return LZMA_OK;
}

// ---- the sliced encode (lzma_enc_session_*): one stream encoded in bounded launches
// begin: the stream's match finder over the whole input (match lists are a pure function of
// the input); step: the parser from the saved state up to the first CodeOneBlock
// boundary past the stop (enc_slice.hip), then the range coder over that slice's records from
// the coder state the last slice left (rc.hip, RcArgs::sliced), its final bytes appended to
// the output; save / restore: the state between steps as a host blob, so a later process can
// go on (the caller keeps the output written so far).
constexpr uint32_t kSessMagic = 0x53455A4Cu;   // "LZES"
constexpr uint32_t kBlobMagic = 0x42455A4Cu;   // "LZEB"
struct EncSession {
    uint32_t magic = kSessMagic;
    Ctx* ctx = nullptr;
    EncPass P;
    lzma_params params{};
    hipStream_t st = nullptr;
    uint8_t* d_state = nullptr;    // the parser's slice state (enc_slice_state_bytes)
    uint32_t* d_rc = nullptr;      // the coder's state between slices (kRcStateWords)
    size_t state_bytes = 0;
    uint64_t n = 0, in_pos = 0, out_len = 0, out_cap = 0;
    int done = 0, steps = 0;
};
static bool ok_sess(const EncSession* s) { return s && s->magic == kSessMagic && s->ctx; }

// the blob: a header of u64 words, then the parser state (absent once the stream is done)
enum { B_MAGIC, B_VERSION, B_DICT, B_FB, B_MF, B_LCLPPB, B_EOS, B_N, B_IN_POS, B_OUT_LEN, B_DONE, B_STATE_BYTES,
       B_RC, B_WORDS = B_RC + kRcStateWords / 2 };

static void session_free(EncSession* S) {
    if (S->d_state) hipFree(S->d_state);
    if (S->d_rc) hipFree(S->d_rc);
    S->d_state = nullptr;
    S->d_rc = nullptr;
}

static int session_begin(Ctx* ctx, const lzma_params* p, const uint8_t* d_in, uint64_t n, uint8_t* d_out, uint64_t out_cap,
                         hipStream_t st, EncSession** out) {
    if (ctx->dec_pending || ctx->split_state || ctx->rc_pending || ctx->session)
        return ctx->fail(LZMA_E_PARAM, "the context is busy (a decode, split encode or session in flight)");
    Derived d;
    if (derive(*p, d) != LZMA_OK) return ctx->fail(LZMA_E_PARAM, "invalid lzma_params");
    if (n >= (1ull << 31)) return ctx->fail(LZMA_E_PARAM, "stream >= 2 GiB");
    if (out_cap < lzma_enc_bound(n)) return ctx->fail(LZMA_E_PARAM, "out_cap below lzma_enc_bound(n)");
    EncSession* S = new (std::nothrow) EncSession;
    if (!S) return ctx->fail(LZMA_E_NOMEM, "session");
    S->ctx = ctx; S->params = *p; S->st = st; S->n = n; S->out_cap = out_cap;
    const uint64_t offs[2] = {0, n}, oofs[2] = {0, out_cap};
    EncPass& P = S->P;
    pass_plan(ctx, P, d, d_in, offs, 0, 1, d_out, oofs, false);
    P.slot = ctx->live[1].n > ctx->live[0].n ? 1 : 0;
    int rc;
    if ((rc = pass_carve(ctx, P)) || (rc = pass_stage(ctx, P, st)) ||
        (rc = mf_front(ctx, P.d, P.inpad, P.d_offs, P.ns, P.total, P.wide, P.w, st)) || (rc = pass_mf_back(ctx, P, st))) {
        delete S;
        return rc;
    }
    S->state_bytes = enc_slice_state_bytes(d);
    ctx->count_alloc(S->state_bytes + kRcStateWords * 4);
    if (hipMalloc(&S->d_state, S->state_bytes) != hipSuccess || hipMalloc(&S->d_rc, kRcStateWords * 4) != hipSuccess) {
        session_free(S);
        delete S;
        return ctx->fail(LZMA_E_NOMEM, "session state");
    }
    ctx->session = S;
    *out = S;
    return LZMA_OK;
}

static int session_step(EncSession* S, uint64_t bytes) {
    Ctx* ctx = S->ctx;
    if (S->done) return LZMA_OK;
    EncPass& P = S->P;
    hipStream_t st = S->st;
    const uint64_t stop = std::min<uint64_t>(S->n, S->in_pos + std::max<uint64_t>(bytes, 1));
    P.slice_state = S->d_state;
    P.slice_stop = (uint32_t)stop;
    P.slice_resume = S->in_pos > 0 ? 1u : 0u;
    int rc;
    if ((rc = pass_parse(ctx, P, st))) return rc;
    // the parser's verdict and where it stopped: the coder's flush depends on it
    uint64_t* pw = ctx->pin.as<uint64_t>();
    HIPCHK(hipMemcpyAsync(pw, S->d_state, SS_WORDS * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(pw + SS_WORDS / 2, P.d_status, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(pw + SS_WORDS / 2 + 1, P.d_lens, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint32_t* sc = (const uint32_t*)pw;
    const int32_t pstat = *(const int32_t*)(pw + SS_WORDS / 2);
    if (pstat != LZMA_OK)
        return ctx->fail(pstat, "sliced parse: consistency check tripped (%llx)", (unsigned long long)pw[SS_WORDS / 2 + 1]);
    if (sc[SS_MAGIC] != kSliceMagic) return ctx->fail(LZMA_E_INTERNAL, "sliced parse left no state");
    const uint64_t now_pos = sc[SS_NOW_POS];
    const int done = sc[SS_DONE] != 0;
    if (now_pos < S->in_pos || now_pos > S->n || (!done && now_pos < stop))
        return ctx->fail(LZMA_E_INTERNAL, "sliced parse stopped at %llu", (unsigned long long)now_pos);
    // the coder over this slice's records, appended at out_len
    const uint64_t oo[2] = {S->out_len, S->out_cap};
    memcpy(pw, oo, 16);
    HIPCHK(hipMemcpyAsync(P.d_oofs, pw, 16, hipMemcpyHostToDevice, st));
    RcArgs ra{};
    ra.sliced = 1;
    ra.flush = done ? 1u : 0u;
    ra.init_state = S->steps > 0 ? S->d_rc : nullptr;
    ra.end_state = S->d_rc;
    if ((rc = pass_rc(ctx, P, P.d_rofs, P.d_rlens, P.d_order, P.d_status, P.d_oofs, P.d_lens, P.d_seg, st, &ra))) return rc;
    HIPCHK(hipMemcpyAsync(pw + 2, P.d_lens, 8, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(pw + 3, P.d_status, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const int32_t cstat = *(const int32_t*)(pw + 3);
    if (cstat != LZMA_OK) return ctx->fail(cstat, "sliced coder failed (%d)", cstat);
    S->out_len += pw[2];
    S->in_pos = now_pos;
    S->done = done;
    S->steps++;
    return LZMA_OK;
}

static int session_save(const EncSession* S, uint8_t* blob, uint64_t cap, uint64_t* len) {
    Ctx* ctx = S->ctx;
    const uint64_t sb = S->done ? 0 : S->state_bytes;
    const uint64_t need = B_WORDS * 8 + sb;
    if (len) *len = need;
    if (!blob) return LZMA_OK;   // size query
    if (cap < need) return ctx->fail(LZMA_E_OVERFLOW, "blob capacity %llu < %llu", (unsigned long long)cap, (unsigned long long)need);
    uint64_t h[B_WORDS] = {};
    h[B_MAGIC] = kBlobMagic; h[B_VERSION] = 1;
    h[B_DICT] = (uint32_t)S->params.dict_size; h[B_FB] = (uint32_t)S->params.fb; h[B_MF] = (uint32_t)S->params.mf;
    h[B_LCLPPB] = (uint64_t)S->params.lc | ((uint64_t)S->params.lp << 8) | ((uint64_t)S->params.pb << 16);
    h[B_EOS] = (uint32_t)S->params.eos; h[B_N] = S->n; h[B_IN_POS] = S->in_pos; h[B_OUT_LEN] = S->out_len;
    h[B_DONE] = (uint64_t)S->done; h[B_STATE_BYTES] = sb;
    uint32_t rcw[kRcStateWords] = {};
    if (S->steps > 0) {
        HIPCHK(hipMemcpy(rcw, S->d_rc, sizeof rcw, hipMemcpyDeviceToHost));
    }
    memcpy(&h[B_RC], rcw, sizeof rcw);
    memcpy(blob, h, sizeof h);
    if (sb) HIPCHK(hipMemcpy(blob + sizeof h, S->d_state, sb, hipMemcpyDeviceToHost));
    return LZMA_OK;
}

static int session_restore(EncSession* S, const uint8_t* blob, uint64_t len) {
    Ctx* ctx = S->ctx;
    if (S->steps > 0) return ctx->fail(LZMA_E_PARAM, "restore: the session has already stepped");
    uint64_t h[B_WORDS];
    if (!blob || len < sizeof h) return ctx->fail(LZMA_E_PARAM, "restore: blob too short");
    memcpy(h, blob, sizeof h);
    const lzma_params& p = S->params;
    if (h[B_MAGIC] != kBlobMagic || h[B_VERSION] != 1) return ctx->fail(LZMA_E_PARAM, "restore: not a session blob");
    if (h[B_DICT] != (uint32_t)p.dict_size || h[B_FB] != (uint32_t)p.fb || h[B_MF] != (uint32_t)p.mf ||
        h[B_LCLPPB] != ((uint64_t)p.lc | ((uint64_t)p.lp << 8) | ((uint64_t)p.pb << 16)) || h[B_EOS] != (uint32_t)p.eos ||
        h[B_N] != S->n)
        return ctx->fail(LZMA_E_PARAM, "restore: the blob is of other parameters or another stream length");
    const uint64_t sb = h[B_STATE_BYTES];
    if ((h[B_DONE] == 0 && sb != S->state_bytes) || len < sizeof h + sb || h[B_IN_POS] > S->n || h[B_OUT_LEN] > S->out_cap)
        return ctx->fail(LZMA_E_PARAM, "restore: inconsistent blob");
    if (h[B_IN_POS] == 0) return LZMA_OK;   // saved before the first step: nothing to restore
    uint32_t rcw[kRcStateWords];
    memcpy(rcw, &h[B_RC], sizeof rcw);
    HIPCHK(hipMemcpy(S->d_rc, rcw, sizeof rcw, hipMemcpyHostToDevice));
    if (sb) HIPCHK(hipMemcpy(S->d_state, blob + sizeof h, sb, hipMemcpyHostToDevice));
    S->in_pos = h[B_IN_POS];
    S->out_len = h[B_OUT_LEN];
    S->done = (int)h[B_DONE];
    S->steps = 1;   // the coder goes on from the blob's state
    return LZMA_OK;
}

}  // namespace lzg

using namespace lzg;

extern "C" {

const char* lzma_version(void) { return "lzma-mi355x 0.1 (gfx950)"; }

int lzma_params_default(lzma_params* p) {   // Encoder field defaults, Encoder.java:135-172
    if (!p) return LZMA_E_PARAM;
    p->dict_size = 1 << 22;
    p->fb = 32;
    p->mf = 1;
    p->lc = 3;
    p->lp = 0;
    p->pb = 2;
    p->eos = 0;
    return LZMA_OK;
}

int lzma_params_check(const lzma_params* p) {
    if (!p) return LZMA_E_PARAM;
    Derived d;
    return derive(*p, d);
}

int lzma_write_props(const lzma_params* p, uint8_t out[5]) {   // Encoder.java:1079-1085
    if (!p || !out) return LZMA_E_PARAM;
    out[0] = (uint8_t)((p->pb * 5 + p->lp) * 9 + p->lc);
    for (int i = 0; i < 4; i++) out[1 + i] = (uint8_t)((uint32_t)p->dict_size >> (8 * i));
    return LZMA_OK;
}

int lzma_read_props(const uint8_t in[5], lzma_params* p) {   // Decoder.java:303-318
    if (!in || !p) return LZMA_E_PARAM;
    uint32_t v = in[0];
    int lc = (int)(v % 9), rem = (int)(v / 9), lp = rem % 5, pb = rem / 5;
    int32_t dict = (int32_t)((uint32_t)in[1] | ((uint32_t)in[2] << 8) | ((uint32_t)in[3] << 16) | ((uint32_t)in[4] << 24));
    if (lc > 8 || lp > 4 || pb > 4) return LZMA_E_PARAM;   // SetLcLpPb :172-182
    if (dict < 0) return LZMA_E_PARAM;                      // SetDictionarySize :160-170
    p->lc = lc; p->lp = lp; p->pb = pb; p->dict_size = dict;
    p->fb = 32; p->mf = 1; p->eos = 0;
    return LZMA_OK;
}

uint64_t lzma_enc_bound(uint64_t n) { return n + n / 8 + 4096; }

uint64_t lzma_visible_on_error(uint32_t dict_size, uint64_t decoded_len) {   // OutWindow.Flush at whole windows
    const uint64_t dict = (int32_t)dict_size < 1 ? 1 : dict_size;                // Decoder.SetDictionarySize :160-170
    const uint64_t w = dict > 4096 ? dict : 4096;                                // Decoder.java:167
    return decoded_len / w * w;
}

int lzma_ctx_create(int device, lzma_ctx** out) {
    if (!out) return LZMA_E_PARAM;
    *out = nullptr;
    int rc = check_device(nullptr);
    if (rc) return rc;
    if (hipSetDevice(device) != hipSuccess) return LZMA_E_DEVICE;
    lzma_ctx* c = new (std::nothrow) lzma_ctx();
    if (!c) return LZMA_E_NOMEM;
    c->device = device;
    {
        std::lock_guard<std::mutex> g(g_ctx_lock);
        g_live_ctx.insert(c);
    }
    *out = c;
    return LZMA_OK;
}

void lzma_ctx_destroy(lzma_ctx* ctx) {
    if (!ok_ctx(ctx)) return;
    {
        std::lock_guard<std::mutex> g(g_ctx_lock);
        g_live_ctx.erase(ctx);
        for (Ctx* o : g_live_ctx)
            if (o->fence == ctx) o->fence = nullptr;   // an encoder fenced on this decoder: no fence any more
    }
    hipSetDevice(ctx->device);
    if (ctx->session) lzma_enc_session_end((lzma_enc_session*)ctx->session);   // its buffers are the context's
    ctx->resolve_timings();
    for (auto e : ctx->free_events) hipEventDestroy(e);
    if (ctx->dec_pending) hipEventSynchronize(ctx->dec_done);
    if (ctx->dec_done) hipEventDestroy(ctx->dec_done);
    for (int q = 0; q < ctx->rc_pending; q++) hipEventSynchronize(ctx->rc_done[ctx->rc_slot[q]]);
    if (ctx->split_state) hipDeviceSynchronize();   // a staged pass's match finder or walk may still run
    for (int k = 0; k < 2; k++) {
        if (ctx->rc_done[k]) hipEventDestroy(ctx->rc_done[k]);
        if (ctx->parse_done[k]) hipEventDestroy(ctx->parse_done[k]);
        ctx->split_recs[k].release();
        ctx->split_coder[k].release();
        ctx->pin_rc[k].release();
        if (ctx->walk_done[k]) hipEventDestroy(ctx->walk_done[k]);
        if (ctx->cnt_done[k]) hipEventDestroy(ctx->cnt_done[k]);
        delete ctx->split_pass[k];
        ctx->live[k].release();
    }
    if (ctx->rc_stream) hipStreamDestroy(ctx->rc_stream);
    if (ctx->walk_stream) hipStreamDestroy(ctx->walk_stream);
    if (ctx->parse_start) hipEventDestroy(ctx->parse_start);

    if (ctx->dec_host) hipHostFree(ctx->dec_host);
    if (ctx->arena) hipFree(ctx->arena);
    if (ctx->litbuf) hipFree(ctx->litbuf);
    if (ctx->tmp) hipFree(ctx->tmp);
    ctx->io_in.release(); ctx->io_out.release(); ctx->io_pack.release(); ctx->io_offs.release();
    ctx->pin.release(); ctx->pin_mf.release();
    ctx->magic = 0;
    delete ctx;
}

const char* lzma_last_error(const lzma_ctx* ctx) { return ok_ctx(ctx) ? ctx->err.c_str() : "null or invalid context"; }

int lzma_ctx_set_batch_bytes(lzma_ctx* ctx, uint64_t bytes) {
    if (!ok_ctx(ctx) || bytes < 4096) return LZMA_E_PARAM;
    ctx->batch_bytes = bytes;
    return LZMA_OK;
}

int lzma_ctx_set_timing(lzma_ctx* ctx, int on) {
    if (!ok_ctx(ctx)) return LZMA_E_PARAM;
    ctx->timing = on != 0;
    return LZMA_OK;
}

int lzma_ctx_timings(lzma_ctx* ctx, const char** names, double* ms, int64_t* launches, int cap) {
    if (!ok_ctx(ctx)) return LZMA_E_PARAM;
    hipSetDevice(ctx->device);
    ctx->resolve_timings();
    int i = 0;
    for (auto& kv : ctx->acc) {
        if (i >= cap) break;
        if (names) names[i] = kv.first.c_str();
        if (ms) ms[i] = kv.second.ms;
        if (launches) launches[i] = kv.second.n;
        i++;
    }
    return i;
}

int lzma_ctx_stats(const lzma_ctx* ctx, uint64_t* allocations, uint64_t* alloc_bytes, uint64_t* device_syncs) {
    if (!ok_ctx(ctx)) return LZMA_E_PARAM;
    uint64_t n = ctx->stat_allocs, b = ctx->stat_alloc_bytes;
    auto add = [&](uint64_t k, uint64_t kb) { n += k; b += kb; };
    for (const DevBuf* d : {&ctx->io_in, &ctx->io_out, &ctx->io_pack, &ctx->io_offs, &ctx->live[0], &ctx->live[1],
                            &ctx->split_recs[0], &ctx->split_recs[1], &ctx->split_coder[0], &ctx->split_coder[1]})
        add(d->allocs, d->alloc_bytes);
    for (const HostBuf* h : {&ctx->pin, &ctx->pin_mf, &ctx->pin_rc[0], &ctx->pin_rc[1]}) add(h->allocs, h->alloc_bytes);
    if (allocations) *allocations = n;
    if (alloc_bytes) *alloc_bytes = b;
    if (device_syncs) *device_syncs = ctx->stat_device_syncs;
    return LZMA_OK;
}

void lzma_ctx_reset_timings(lzma_ctx* ctx) {
    if (!ok_ctx(ctx)) return;
    ctx->resolve_timings();
    ctx->acc.clear();
}

int lzma_enc_batch_dev(lzma_ctx* ctx, const lzma_params* p, const uint8_t* d_in, const uint64_t* h_offs, int nstreams,
                       uint8_t* d_out, const uint64_t* h_out_offs, uint64_t* h_out_lens, void* hip_stream) {
    if (!ok_ctx(ctx) || !p || !h_offs || !h_out_offs || !h_out_lens) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    return encode_batch_dev(ctx, p, d_in, h_offs, nstreams, d_out, h_out_offs, h_out_lens, (hipStream_t)hip_stream);
}

int lzma_enc_stage_dev(lzma_ctx* ctx, const lzma_params* p, const uint8_t* d_in, const uint64_t* h_offs, int nstreams,
                       uint8_t* d_out, const uint64_t* h_out_offs, void* hip_stream) {
    if (!ok_ctx(ctx) || !p || !h_offs || !h_out_offs) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    return enc_stage_dev(ctx, p, d_in, h_offs, nstreams, d_out, h_out_offs, (hipStream_t)hip_stream);
}

int lzma_enc_parse_dev_async(lzma_ctx* ctx, void* hip_stream) {
    if (!ok_ctx(ctx)) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    return enc_parse_dev_async(ctx, (hipStream_t)hip_stream);
}

int lzma_enc_parse_dev_wait(lzma_ctx* ctx, uint64_t* h_out_lens) {
    if (!ok_ctx(ctx) || !h_out_lens) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    return enc_parse_dev_wait(ctx, h_out_lens);
}

int lzma_pack_dev(lzma_ctx* ctx, const uint8_t* d_src, const uint64_t* h_src_offs, const uint64_t* h_lens, int nstreams,
                  uint8_t* d_dst, const uint64_t* h_dst_offs, void* hip_stream) {
    if (!ok_ctx(ctx) || !h_src_offs || !h_lens || !h_dst_offs || nstreams < 0) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    if (nstreams == 0) return LZMA_OK;
    // the pack carves the front of the arena, where a decode in flight keeps its offsets
    // and results (decode_enqueue), and may grow (reallocate) it
    if (ctx->dec_pending) return ctx->fail(LZMA_E_PARAM, "an asynchronous decode is in flight: lzma_dec_batch_dev_wait first");
    if (ctx->split_state || ctx->rc_pending)
        return ctx->fail(LZMA_E_PARAM, "a split encode is in flight on this context: lzma_enc_parse_dev_async / _wait first");
    if (ctx->session) return ctx->fail(LZMA_E_PARAM, "an encode session is open on this context: lzma_enc_session_end first");
    hipSetDevice(ctx->device);
    hipStream_t st = (hipStream_t)hip_stream;
    for (int i = 0; i < nstreams; i++)
        if (h_dst_offs[i + 1] - h_dst_offs[i] != h_lens[i]) return ctx->fail(LZMA_E_PARAM, "dst offsets must be the prefix sum of lens");
    Carver probe(nullptr);
    probe.take<uint64_t>(nstreams + 1);
    probe.take<uint64_t>(nstreams + 1);
    if (!ctx->ensure_arena(probe.off + 4096)) return ctx->fail(LZMA_E_NOMEM, "pack workspace");
    Carver c(ctx->arena);
    uint64_t* d_so = c.take<uint64_t>(nstreams + 1);
    uint64_t* d_do = c.take<uint64_t>(nstreams + 1);
    if (!ctx->pin.ensure((size_t)(nstreams + 1) * 16)) return ctx->fail(LZMA_E_NOMEM, "pinned staging");
    uint64_t* p_so = ctx->pin.as<uint64_t>();
    uint64_t* p_do = p_so + nstreams + 1;
    memcpy(p_so, h_src_offs, (size_t)(nstreams + 1) * 8);
    memcpy(p_do, h_dst_offs, (size_t)(nstreams + 1) * 8);
    HIPCHK(hipMemcpyAsync(d_so, p_so, (nstreams + 1) * 8, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemcpyAsync(d_do, p_do, (nstreams + 1) * 8, hipMemcpyHostToDevice, st));
    {
        TimedLaunch tl(ctx, "pack", st);
        hipLaunchKernelGGL(pack_kernel, dim3(std::min(nstreams, 65535)), dim3(256), 0, st, d_src, d_so, d_do, d_dst, nstreams);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(st));
    return LZMA_OK;
}

int lzma_enc_batch(lzma_ctx* ctx, const lzma_params* p, const uint8_t* in, const uint64_t* offs, int nstreams,
                   uint8_t* out, uint64_t out_cap, uint64_t* out_offs) {
    if (!ok_ctx(ctx) || !p || !offs || !out_offs || nstreams < 0) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    Derived d;
    if (derive(*p, d) != LZMA_OK) return ctx->fail(LZMA_E_PARAM, "invalid lzma_params");
    const uint64_t total = offs[nstreams] - offs[0];
    std::vector<uint64_t> rel(nstreams + 1), cap_offs(nstreams + 1), lens(nstreams), pack(nstreams + 1);
    cap_offs[0] = 0;
    for (int i = 0; i <= nstreams; i++) rel[i] = offs[i] - offs[0];
    for (int i = 0; i < nstreams; i++) cap_offs[i + 1] = cap_offs[i] + lzma_enc_bound(rel[i + 1] - rel[i]);
    // staging buffers persist in the context (grown, never shrunk): no hipMalloc per call
    if (!ctx->io_in.ensure(total + 1) || !ctx->io_out.ensure(cap_offs[nstreams] + 1) ||
        !ctx->io_offs.ensure(16 * ((size_t)nstreams + 1)))
        return ctx->fail(LZMA_E_NOMEM, "device staging buffers");
    uint8_t* d_in = ctx->io_in.as<uint8_t>();
    uint8_t* d_out = ctx->io_out.as<uint8_t>();
    uint64_t* d_co = ctx->io_offs.as<uint64_t>();
    uint64_t* d_po = d_co + nstreams + 1;
    hipStream_t st = nullptr;
    if (total) HIPCHK(hipMemcpy(d_in, in + offs[0], total, hipMemcpyHostToDevice));
    int rc = encode_batch_dev(ctx, p, d_in, rel.data(), nstreams, d_out, cap_offs.data(), lens.data(), st);
    if (rc) return rc;
    pack[0] = 0;
    for (int i = 0; i < nstreams; i++) pack[i + 1] = pack[i] + lens[i];
    if (pack[nstreams] > out_cap)
        return ctx->fail(LZMA_E_OVERFLOW, "out_cap %llu < %llu", (unsigned long long)out_cap, (unsigned long long)pack[nstreams]);
    if (!ctx->io_pack.ensure(pack[nstreams] + 1)) return ctx->fail(LZMA_E_NOMEM, "pack buffer");
    uint8_t* d_pack = ctx->io_pack.as<uint8_t>();
    HIPCHK(hipMemcpy(d_co, cap_offs.data(), (nstreams + 1) * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_po, pack.data(), (nstreams + 1) * 8, hipMemcpyHostToDevice));
    if (nstreams > 0) hipLaunchKernelGGL(pack_kernel, dim3(std::min(nstreams, 65535)), dim3(256), 0, st, d_out, d_co, d_po, d_pack, nstreams);
    HIPCHK(hipGetLastError());
    if (pack[nstreams]) HIPCHK(hipMemcpy(out, d_pack, pack[nstreams], hipMemcpyDeviceToHost));
    for (int i = 0; i <= nstreams; i++) out_offs[i] = pack[i];
    return LZMA_OK;
}

int lzma_match_lists(lzma_ctx* ctx, const lzma_params* p, const uint8_t* in, const uint64_t* offs, int nstreams,
                     uint32_t* counts, uint32_t* main_len, uint32_t* lens, uint32_t* dists, uint64_t cap,
                     uint64_t* total_pairs) {
    if (!ok_ctx(ctx) || !p || !offs || nstreams < 0 || !counts || !main_len || !total_pairs) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    Derived d;
    if (derive(*p, d) != LZMA_OK) return ctx->fail(LZMA_E_PARAM, "invalid lzma_params");
    *total_pairs = 0;
    if (nstreams == 0) return LZMA_OK;
    const uint64_t total = offs[nstreams] - offs[0];
    if (total >= (1ull << 31)) return ctx->fail(LZMA_E_PARAM, "match-list dump is limited to one pass (< 2 GiB)");
    // one pass: the match finder's 32-bit hash2/hash3 sort keys hold the stream index in the bits above the
    // hash (runtime.h MfArgs), valid for at most kMaxStreamsPerPass streams
    if (nstreams > kMaxStreamsPerPass)
        return ctx->fail(LZMA_E_PARAM, "match-list dump is limited to %d streams per call", kMaxStreamsPerPass);
    std::vector<uint64_t> rel(nstreams + 1), oo(nstreams + 1, 0), lens_h(nstreams);
    std::vector<int32_t> status(nstreams);
    for (int i = 0; i <= nstreams; i++) {
        rel[i] = offs[i] - offs[0];
        if (i && rel[i] < rel[i - 1]) return ctx->fail(LZMA_E_PARAM, "offsets not monotone");
    }
    if (!ctx->io_in.ensure(total + 1)) return ctx->fail(LZMA_E_NOMEM, "device input");
    uint8_t* d_in = ctx->io_in.as<uint8_t>();
    if (total) HIPCHK(hipMemcpy(d_in, in + offs[0], total, hipMemcpyHostToDevice));
    MatchDump dump;
    int rc = encode_pass(ctx, d, d_in, rel.data(), 0, nstreams, nullptr, oo.data(), lens_h.data(), status.data(),
                         nullptr, &dump);
    if (rc) return rc;
    uint64_t k = 0;
    const uint32_t rb = rec_bytes(dump.wide), psz = dump.wide ? 8 : 4;
    for (uint64_t g = 0; g < total; g++) {
        const uint8_t* rec = &dump.recs[g * rb];
        uint32_t info;
        memcpy(&info, rec + rb - 16, 4);   // the record's last vector
        const uint32_t cnt = info & 0xFFFFu;
        counts[g] = cnt;
        main_len[g] = info >> 16;
        for (uint32_t j = 0; j < cnt; j++, k++) {
            uint64_t pr;
            const uint8_t* src;
            if (j < (uint32_t)kInlinePairs) {
                src = rec + j * psz;
            } else {
                const uint64_t idx = (uint64_t)dump.ovf_off[g] * dump.stride + j - kInlinePairs;
                if ((idx + 1) * psz > dump.ovf.size()) return ctx->fail(LZMA_E_INTERNAL, "pair index out of range");
                src = &dump.ovf[idx * psz];
            }
            if (dump.wide) {
                memcpy(&pr, src, 8);
            } else {
                uint32_t v;
                memcpy(&v, src, 4);
                pr = ((uint64_t)(v >> 23) << 32) | (v & 0x7FFFFFu);
            }
            if (k < cap && lens && dists) { lens[k] = (uint32_t)(pr >> 32); dists[k] = (uint32_t)pr; }
        }
    }
    *total_pairs = k;
    if (k > cap) return ctx->fail(LZMA_E_OVERFLOW, "%llu pairs > cap %llu", (unsigned long long)k, (unsigned long long)cap);
    return LZMA_OK;
}

int lzma_enc_session_begin(lzma_ctx* ctx, const lzma_params* p, const uint8_t* d_in, uint64_t n, uint8_t* d_out,
                           uint64_t out_cap, void* hip_stream, lzma_enc_session** out) {
    if (!ok_ctx(ctx) || !p || !out) return LZMA_E_PARAM;
    *out = nullptr;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    EncSession* S = nullptr;
    int rc = session_begin(ctx, p, d_in, n, d_out, out_cap, (hipStream_t)hip_stream, &S);
    if (rc == LZMA_OK) *out = (lzma_enc_session*)S;
    return rc;
}

int lzma_enc_session_begin_host(lzma_ctx* ctx, const lzma_params* p, const uint8_t* in, uint64_t n,
                                lzma_enc_session** out) {
    if (!ok_ctx(ctx) || !p || !out || (n && !in)) return LZMA_E_PARAM;
    *out = nullptr;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    if (ctx->dec_pending || ctx->split_state || ctx->rc_pending || ctx->session)
        return ctx->fail(LZMA_E_PARAM, "the context is busy (a decode, split encode or session in flight)");
    const uint64_t cap = lzma_enc_bound(n);
    // the context's staging buffers (grown, never shrunk): no allocation per call once sized
    if (!ctx->io_in.ensure(n + 1) || !ctx->io_out.ensure(cap + 1)) return ctx->fail(LZMA_E_NOMEM, "device staging buffers");
    if (n) HIPCHK(hipMemcpy(ctx->io_in.as<uint8_t>(), in, n, hipMemcpyHostToDevice));
    EncSession* S = nullptr;
    int rc = session_begin(ctx, p, ctx->io_in.as<uint8_t>(), n, ctx->io_out.as<uint8_t>(), cap, nullptr, &S);
    if (rc == LZMA_OK) *out = (lzma_enc_session*)S;
    return rc;
}

int lzma_enc_session_output(const lzma_enc_session* s, uint64_t from, uint8_t* dst, uint64_t len) {
    const EncSession* S = (const EncSession*)s;
    if (!ok_sess(S) || (len && !dst)) return LZMA_E_PARAM;
    Ctx* ctx = S->ctx;
    if (from > S->out_len || len > S->out_len - from)
        return ctx->fail(LZMA_E_PARAM, "output [%llu, +%llu) is not final yet (%llu bytes are)", (unsigned long long)from,
                         (unsigned long long)len, (unsigned long long)S->out_len);
    hipSetDevice(ctx->device);
    if (len) HIPCHK(hipMemcpy(dst, S->P.d_out + from, len, hipMemcpyDeviceToHost));
    return LZMA_OK;
}

int lzma_enc_session_step(lzma_enc_session* s, uint64_t bytes, uint64_t* in_pos, uint64_t* out_len, int* done) {
    EncSession* S = (EncSession*)s;
    if (!ok_sess(S)) return LZMA_E_PARAM;
    hipSetDevice(S->ctx->device);
    int rc = session_step(S, bytes);
    if (in_pos) *in_pos = S->in_pos;
    if (out_len) *out_len = S->out_len;
    if (done) *done = S->done;
    return rc;
}

int lzma_enc_session_save(const lzma_enc_session* s, uint8_t* blob, uint64_t cap, uint64_t* len) {
    const EncSession* S = (const EncSession*)s;
    if (!ok_sess(S)) return LZMA_E_PARAM;
    hipSetDevice(S->ctx->device);
    return session_save(S, blob, cap, len);
}

int lzma_enc_session_restore(lzma_enc_session* s, const uint8_t* blob, uint64_t len) {
    EncSession* S = (EncSession*)s;
    if (!ok_sess(S)) return LZMA_E_PARAM;
    hipSetDevice(S->ctx->device);
    return session_restore(S, blob, len);
}

void lzma_enc_session_end(lzma_enc_session* s) {
    EncSession* S = (EncSession*)s;
    if (!ok_sess(S)) return;
    hipSetDevice(S->ctx->device);
    hipStreamSynchronize(S->st);
    session_free(S);
    if (S->ctx->session == S) S->ctx->session = nullptr;
    S->magic = 0;
    delete S;
}

int lzma_encode(lzma_ctx* ctx, const lzma_params* p, const uint8_t* in, uint64_t n, uint8_t* out, uint64_t out_cap,
                uint64_t* out_len) {
    uint64_t offs[2] = {0, n}, oo[2] = {0, 0};
    int rc = lzma_enc_batch(ctx, p, in, offs, 1, out, out_cap, oo);
    if (rc == LZMA_OK && out_len) *out_len = oo[1];
    return rc;
}

int lzma_dec_batch_dev(lzma_ctx* ctx, const uint8_t props[5], const uint8_t* d_in, const uint64_t* h_in_offs, int nstreams,
                       const int64_t* h_out_sizes, uint8_t* d_out, const uint64_t* h_out_offs, uint64_t* h_out_lens,
                       int32_t* h_status, void* hip_stream) {
    if (!ok_ctx(ctx) || !props || !h_in_offs || !h_out_sizes || !h_out_offs || !h_out_lens || !h_status) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    return decode_batch_dev(ctx, props, d_in, h_in_offs, nstreams, h_out_sizes, d_out, h_out_offs, h_out_lens, h_status,
                            (hipStream_t)hip_stream);
}

int lzma_dec_batch_dev_async(lzma_ctx* ctx, const uint8_t props[5], const uint8_t* d_in, const uint64_t* h_in_offs,
                             int nstreams, const int64_t* h_out_sizes, uint8_t* d_out, const uint64_t* h_out_offs,
                             void* hip_stream) {
    if (!ok_ctx(ctx) || !props || !h_in_offs || !h_out_sizes || !h_out_offs) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    return decode_batch_dev_async(ctx, props, d_in, h_in_offs, nstreams, h_out_sizes, d_out, h_out_offs,
                                  (hipStream_t)hip_stream);
}

int lzma_dec_batch_dev_wait(lzma_ctx* ctx, uint64_t* h_out_lens, int32_t* h_status) {
    if (!ok_ctx(ctx)) return LZMA_E_PARAM;
    hipSetDevice(ctx->device);
    return decode_batch_dev_wait(ctx, h_out_lens, h_status);
}

int lzma_ctx_set_parse_fence(lzma_ctx* ctx, const lzma_ctx* dec_ctx) {
    if (!ok_ctx(ctx) || (dec_ctx && !ok_ctx(dec_ctx)) || dec_ctx == ctx) return LZMA_E_PARAM;
    if (dec_ctx && dec_ctx->device != ctx->device) return ctx->fail(LZMA_E_PARAM, "parse fence on another device");
    ctx->fence = dec_ctx;
    return LZMA_OK;
}

int lzma_dec_batch(lzma_ctx* ctx, const uint8_t props[5], const uint8_t* in, const uint64_t* in_offs, int nstreams,
                   const int64_t* out_sizes, uint8_t* out, const uint64_t* out_offs, uint64_t* out_lens, int32_t* status) {
    if (!ok_ctx(ctx) || !props || !in_offs || !out_sizes || !out_offs || !out_lens || !status || nstreams < 0) return LZMA_E_PARAM;
    if (check_device(ctx)) return LZMA_E_NODEVICE;
    hipSetDevice(ctx->device);
    const uint64_t tin = in_offs[nstreams] - in_offs[0];
    const uint64_t tout = out_offs[nstreams] - out_offs[0];
    std::vector<uint64_t> rin(nstreams + 1), rout(nstreams + 1);
    for (int i = 0; i <= nstreams; i++) { rin[i] = in_offs[i] - in_offs[0]; rout[i] = out_offs[i] - out_offs[0]; }
    // staging buffers persist in the context (grown, never shrunk): no hipMalloc per call
    if (!ctx->io_in.ensure(tin + 1) || !ctx->io_out.ensure(tout + 1)) return ctx->fail(LZMA_E_NOMEM, "device buffers");
    uint8_t* d_in = ctx->io_in.as<uint8_t>();
    uint8_t* d_out = ctx->io_out.as<uint8_t>();
    if (tin) HIPCHK(hipMemcpy(d_in, in + in_offs[0], tin, hipMemcpyHostToDevice));
    int rc = decode_batch_dev(ctx, props, d_in, rin.data(), nstreams, out_sizes, d_out, rout.data(), out_lens, status, nullptr);
    if (rc == LZMA_OK && tout) {
        if (nstreams > 16) {   // one copy of the whole layout (bytes past a stream's length are capacity)
            HIPCHK(hipMemcpy(out + out_offs[0], d_out, tout, hipMemcpyDeviceToHost));
        } else {
            for (int i = 0; i < nstreams; i++) {
                uint64_t L = std::min<uint64_t>(out_lens[i], rout[i + 1] - rout[i]);
                if (L) HIPCHK(hipMemcpy(out + out_offs[i], d_out + rout[i], L, hipMemcpyDeviceToHost));
            }
        }
    }
    return rc;
}

int lzma_decode(lzma_ctx* ctx, const uint8_t props[5], const uint8_t* in, uint64_t n, int64_t out_size, uint8_t* out,
                uint64_t out_cap, uint64_t* out_len) {
    uint64_t io[2] = {0, n}, oo[2] = {0, out_cap}, len = 0;
    int32_t st = 0;
    int rc = lzma_dec_batch(ctx, props, in, io, 1, &out_size, out, oo, &len, &st);
    if (out_len) *out_len = len;
    if (rc) return rc;
    return st;
}

// LzmaBench.CBenchRandomGenerator (LzmaBench.java:15-127): MWC RNG, bit
// reservoir, literal with p = 1/2 else a short-offset copy.
void lzma_bench_generate(uint8_t* buf, uint64_t size) {
    uint32_t A1 = 362436069u, A2 = 521288629u;   // CRandomGenerator.Init :23-26
    uint32_t value = 0;
    int num_bits = 0;
    auto rnd32 = [&]() -> uint32_t {   // GetRnd :28-32
        A1 = 36969u * (A1 & 0xffffu) + (A1 >> 16);
        A2 = 18000u * (A2 & 0xffffu) + (A2 >> 16);
        return (A1 << 16) ^ A2;
    };
    auto get = [&](int nb) -> uint32_t {   // CBitRandomGenerator.GetRnd :45-60
        uint32_t result;
        if (num_bits > nb) {
            result = value & ((1u << nb) - 1);
            value >>= nb;
            num_bits -= nb;
            return result;
        }
        nb -= num_bits;
        result = nb >= 32 ? 0 : (value << nb);
        value = rnd32();
        result |= value & (nb >= 32 ? 0xFFFFFFFFu : ((1u << nb) - 1));
        value = nb >= 32 ? 0 : (value >> nb);
        num_bits = 32 - nb;
        return result;
    };
    auto log_bits = [&](int nb) -> uint32_t { uint32_t len = get(nb); return get((int)len); };   // :84-87
    uint64_t pos = 0;
    uint32_t rep0 = 1;
    while (pos < size) {   // Generate :104-127
        if (get(1) == 0 || pos < 1) {
            buf[pos++] = (uint8_t)get(8);
        } else {
            uint32_t len;
            if (get(3) == 0) {
                len = 1 + get(1 + (int)get(2));
            } else {
                do {
                    if (get(1) == 0) {
                        rep0 = log_bits(4);
                    } else {   // Java evaluates left to right: high part first
                        uint32_t hi = log_bits(4);
                        rep0 = (hi << 10) | get(10);
                    }
                } while (rep0 >= pos);
                rep0++;
                len = 2 + get(2 + (int)get(2));
            }
            for (uint32_t i = 0; i < len && pos < size; i++, pos++) buf[pos] = buf[pos - rep0];
        }
    }
}

}  // extern "C"
