// rc.hip -- the range coder of src/main/java/SevenZip/Compression/RangeCoder/
// Encoder.java (RangeEncoder.java:18-87) run over the parser's coder records.
//
// enc.hip emits one 16-bit record per binary decision of the symbol coder:
// the probability before its update (11 bits) and the bit (bit 11); a record
// with probability 0 is a direct bit (EncodeDirectBits, :56-67). The coder's
// arithmetic never feeds back into the parse, so it runs here, after the
// parse, one LANE per stream: the serial chain of every stream runs on the
// vector unit (64 streams per wave instruction) instead of the single scalar
// unit of a CU that the 16 parser waves already share.
//
// A stream's chain is serial, so the kernel time is one stream's chain
// latency. The step is therefore straight-line code over a block of 64
// records (no branches: the compiler interleaves the next record's range
// update with this record's low/output bookkeeping):
//   * `low` is 32 bits plus a carry bit: after ShiftLow low < 2^32, and the
//     bounds added before the next ShiftLow sum to less than the range;
//   * output bytes go to a per-lane LDS ring with unconditional writes: the
//     cache byte at outpos and one pending 0xFF/0x00 byte after it (positions
//     >= outpos are not final yet, so a write there that turns out not to be
//     an emission is overwritten later);
//   * after each block the ring goes to HBM as 18 aligned dwords into the
//     stream's own record region, which serves as the output staging area: a
//     record is 2 bytes and makes at most one byte, so output position k is
//     always far behind the records still to be read; rc_merge_kernel then
//     assembles each stream's bytes in the caller's output layout;
//   * a pending run of two or more 0xFF bytes (cacheSize > 2 at an emission,
//     about once per 2^16 shifts) only sets a flag: lanes that raised it replay
//     the block from the saved state with the exact reference step, writing
//     straight to HBM.
#include "lzma_common.h"
#include "runtime.h"

namespace lzg {

constexpr int kRcRing = 72;             // bytes per lane: a block starts <= 3 bytes past its base and emits <= 66
constexpr int kRcStride = kRcRing + 4;  // 19 dwords: lane rings start in distinct LDS banks
constexpr int kRcLanes = 64;

struct RcState {
    uint32_t lo, carry, range, cache, cache_size;
    uint32_t outpos;   // streams < 2 GiB: outputs < 4 GiB
};

struct RcLane : RcState {
    uint8_t* stage;    // output staging: the stream's record region
    uint8_t* ring;     // this lane's ring: byte k is output position base + k

    uint32_t tailw;    // the staged dword holding position outpos - 1 (kept by put)

    // ---- exact reference step (replay and stream tail): bytes straight to the staging area
    __device__ __forceinline__ void put(uint32_t b) {
        const uint32_t sh = (outpos & 3u) * 8;
        tailw = (tailw & ~(0xFFu << sh)) | ((b & 0xFFu) << sh);
        stage[outpos++] = (uint8_t)b;
    }
    __device__ __forceinline__ void shift_low() {   // RangeEncoder.ShiftLow (:73-87)
        if (carry != 0 || lo < 0xFF000000u) {
            uint32_t temp = cache;
#pragma unroll 1
            do { put((temp + carry) & 0xFFu); temp = 0xFF; } while (--cache_size != 0);
            cache = lo >> 24;
        }
        cache_size++;
        lo = (lo & 0xFFFFFFu) << 8;
        carry = 0;
    }
    // Encode (:38-54) for prob != 0, one EncodeDirectBits step (:56-67) for prob == 0
    __device__ __forceinline__ void step_exact(uint32_t rec) {
        const uint32_t p = rec & 0x7FFu, bit = (rec >> 11) & 1u;
        const uint32_t bound = p ? (range >> 11) * p : range >> 1;
        if (bit) {
            const uint32_t nl = lo + bound;
            carry |= nl < lo;
            lo = nl;
        }
        range = (bit && p) ? range - bound : bound;
        if (range < (1u << 24)) { range <<= 8; shift_low(); }
    }

    // ---- fast step: selects and unconditional ring writes only
    __device__ __forceinline__ void step_fast(uint32_t rec, uint32_t base, bool& flag) {
        const uint32_t p = rec & 0x7FFu;
        const bool bit = (rec & 0x800u) != 0, direct = p == 0;
        const uint32_t bp = (range >> 11) * p, bd = range >> 1;
        const uint32_t bound = direct ? bd : bp;
        const uint32_t r1 = (bit && !direct) ? range - bp : bound;
        const bool norm = r1 < (1u << 24);
        range = norm ? r1 << 8 : r1;
        const uint32_t add = bit ? bound : 0u;
        const uint32_t l = lo + add;
        const uint32_t c = carry + (l < add ? 1u : 0u);   // at most one carry between two ShiftLows
        // ShiftLow when norm: the cache group [outpos, outpos + cache_size) leaves when the
        // carry is known (carry set or the top byte < 0xFF)
        const uint32_t top = l >> 24;
        const bool emit = norm && ((c << 8) | top) != 0xFFu;
        flag |= emit && cache_size > 2;
#ifdef LZG_RC_FORCE_REPLAY
        flag = true;   // test builds: every block takes the exact replay path
#endif
        ring[outpos - base] = (uint8_t)(cache + c);
        ring[outpos - base + 1] = (uint8_t)(0xFFu + c);
        outpos += emit ? cache_size : 0u;
        cache = emit ? top : cache;
        cache_size = emit ? 1u : cache_size + (norm ? 1u : 0u);
        lo = norm ? l << 8 : l;
        carry = norm ? 0u : c;
    }
};

__device__ __forceinline__ uint32_t rec_at(const uint32_t (&w)[32], int k) {
    return (w[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
}

// Segments: a stream's records are cut into kRcSegs runs at multiples of 128 records
// (split_k = min(n, k * seglen)). The range sequence does not depend on low, so one
// cheap range-only pass gives every segment its starting range; the segments are
// then coded independently from low = 0 (8 lanes per stream), and rc_merge_kernel
// adds them up. Why the sum is the reference's output: the coder's bytes are the
// base-256 digits of low, a sum of bound contributions that normalisation shifts
// by whole bytes; a segment started at the window of split_k with low = 0 produces
// exactly its records' contributions, its cache byte at the digit before that
// window. Segment k's bytes begin at pos_k, pos_{k+1} = pos_k + outlen_k + cs_k - 1
// (emitted bytes + pending group = 1 + shifts), and its unfinished digits (cache,
// cs_k - 1 pending 0xFF, the 4 bytes of low, the carry at the last pending digit)
// add into the next segment's first bytes; carries run toward the stream start.
// 128-record multiples: a segment's staged bytes (at most records + 1, plus the ring's
// 72-byte write-back past them) then stay inside its own 2-byte-per-record region
// The sliced encode (RcArgs::sliced) cuts differently: the coder's end state after a slice
// is the end state of its last non-empty segment only if no earlier segment's unfinished
// digits reach that segment's own unfinished digits. Below 2^20 records a slice is one
// segment (segments 1.. are empty); above, the splits round down, so the last segment holds
// at least n / 16 >= 65536 records and emits far more than the 5 digits an earlier
// segment's tail adds into its first bytes (rc_merge_kernel checks it).
__device__ __forceinline__ uint64_t rc_seglen(uint64_t n, bool sliced = false) {
    if (sliced) return n < (1u << 20) ? (n ? n : 1) : (n / (128 * kRcSegs)) * 128;
    return ((n + 128 * kRcSegs - 1) / (128 * kRcSegs)) * 128;
}
__device__ __forceinline__ uint64_t rc_split(uint64_t n, uint64_t seglen, int k) {
    const uint64_t v = (uint64_t)k * seglen;
    return v < n ? v : n;
}

// range-only pass: seg[s][k].range for k = 1 .. kRcSegs - 1, one lane per stream
__global__ void __launch_bounds__(kRcLanes) rc_range_kernel(RcArgs a) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= a.nstreams) return;
    const uint32_t s = a.order[i];
    if (a.status[s] != LZMA_OK) return;
    const uint64_t n = a.rec_lens[s], seglen = rc_seglen(n, a.sliced);
    const uint32_t* r32 = (const uint32_t*)(a.recs + a.rec_offs[s]);
    uint32_t* seg = a.seg + (size_t)s * kRcSegs * kRcSegWords;
    const uint64_t need = rc_split(n, seglen, kRcSegs - 1);   // records before the last split
    uint32_t range = a.init_state ? a.init_state[(size_t)s * kRcStateWords] : 0xFFFFFFFFu;
    seg[0] = range;
    int next = 1;                                            // next split to record
    // Encode / EncodeDirectBits, range only. bit ? range - t*p : t*p (t = range >> 11) is one
    // 24-bit multiply-add, (range & -bit) + t * (bit ? -p : p), exact mod 2^32; the next range
    // is >= 2^17 (t >= 2^13, 31 <= p <= 2017), so it needs the 8-bit shift exactly when its
    // leading-zero count has bit 3 set (8..14)
    auto step = [&](uint32_t rec) {
        const uint32_t p = rec & 0x7FFu;
        const uint32_t bm = 0u - ((rec >> 11) & 1u);
        const int32_t q = (int32_t)((p ^ bm) - bm);
        const uint32_t t = range >> 11;
        const uint32_t r1p = (range & bm) + (uint32_t)((int64_t)(int32_t)t * q);   // |t*q| < 2^32: 24-bit operands, low word kept
        const uint32_t dm = 0u - (uint32_t)(p == 0);   // a direct bit: range >> 1 (a mask, not a branch)
        const uint32_t r1 = r1p ^ ((r1p ^ (range >> 1)) & dm);
        range = r1 << ((uint32_t)__builtin_clz(r1) & 8u);
    };
    const uint64_t nblk = (need + 63) >> 6, full = need >> 6;
    uint32_t cur[32], nxt[32];
    if (nblk) {
#pragma unroll
        for (int j = 0; j < 32; j++) cur[j] = __builtin_nontemporal_load(r32 + j);
    }
    for (uint64_t b = 0; b < nblk; b++) {
        while (next < kRcSegs && rc_split(n, seglen, next) == b * 64) seg[(next++) * kRcSegWords] = range;
        if (b + 1 < nblk) {
#pragma unroll
            for (int j = 0; j < 32; j++) nxt[j] = __builtin_nontemporal_load(r32 + (b + 1) * 32 + j);
        }
        if (b < full) {
#pragma unroll
            for (int k = 0; k < 64; k++) step(rec_at(cur, k));
        } else {
            const uint32_t m = (uint32_t)(need & 63);
#pragma unroll 1
            for (uint32_t k = 0; k < m; k++) step(rec_at(cur, (int)k));
        }
#pragma unroll
        for (int j = 0; j < 32; j++) cur[j] = nxt[j];
    }
    while (next < kRcSegs) seg[(next++) * kRcSegWords] = range;   // splits at `need` (and empty segments)
}

// one lane per (stream, segment): the segment's records from its starting range and
// low = 0; bytes staged at the segment's own record offset, state left in seg[s][k]
__global__ void __launch_bounds__(kRcLanes) rc_kernel(RcArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t rings[kRcLanes * kRcStride / 4];
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= a.nstreams * kRcSegs) return;
    const uint32_t s = a.order[i / kRcSegs];
    const int sk = i % kRcSegs;
    if (a.status[s] != LZMA_OK) return;
    const uint64_t nall = a.rec_lens[s], seglen = rc_seglen(nall, a.sliced);
    const uint64_t r0 = rc_split(nall, seglen, sk);
    const uint64_t n = (sk + 1 < kRcSegs ? rc_split(nall, seglen, sk + 1) : nall) - r0;
    uint16_t* region = a.recs + a.rec_offs[s] + r0;   // 64-record (128-byte) aligned
    uint32_t* seg = a.seg + ((size_t)s * kRcSegs + sk) * kRcSegWords;
    const uint32_t* r32 = (const uint32_t*)region;
    uint32_t* ring32 = rings + threadIdx.x * (kRcStride / 4);
    uint32_t* stage32 = (uint32_t*)region;
    RcLane c;
    c.stage = (uint8_t*)region;
    c.ring = (uint8_t*)ring32;
    c.outpos = 0;
    c.tailw = 0;
    c.lo = 0; c.carry = 0; c.range = seg[0]; c.cache = 0; c.cache_size = 1;   // Init (:18-24) at the segment's range
    if (sk == 0 && a.init_state) {   // a slice of a longer stream: the coder where the last slice left it
        const uint32_t* is = a.init_state + (size_t)s * kRcStateWords;
        c.lo = is[1]; c.carry = is[2]; c.cache = is[3]; c.cache_size = is[4];
    }
    // blocks of 64 records (32 dwords per lane); the next block's loads are issued
    // before this block is coded, so their HBM latency overlaps the coding
    const uint64_t nblk = (n + 63) >> 6, full = n >> 6;
    uint32_t cur[32], nxt[32];
    if (nblk) {
#pragma unroll
        for (int j = 0; j < 32; j++) cur[j] = __builtin_nontemporal_load(r32 + j);
    }
    uint32_t base = 0;   // the ring's first byte is output position base (a multiple of 4)
    for (uint64_t b = 0; b < nblk; b++) {
        if (b + 1 < nblk) {
#pragma unroll
            for (int j = 0; j < 32; j++) nxt[j] = __builtin_nontemporal_load(r32 + (b + 1) * 32 + j);
        }
        if (b < full) {
            // carry the final bytes [nb, outpos) of the last partial dword to the ring start
            const uint32_t nb = c.outpos & ~3u;
            ring32[0] = ring32[(nb - base) >> 2];
            c.tailw = ring32[0];
            base = nb;
            const RcState saved = c;
            bool flag = false;
#pragma unroll
            for (int k = 0; k < 64; k++) c.step_fast(rec_at(cur, k), base, flag);
            if (__builtin_amdgcn_ballot_w64(flag) && flag) {   // rare: replay the block exactly
                (RcState&)c = saved;
#pragma unroll 1
                for (int k = 0; k < 64; k++) c.step_exact(rec_at(cur, k));
                // the ring restarts at the replay's last partial dword (its final bytes: tailw)
                base = c.outpos & ~3u;
                ring32[0] = c.tailw;
            } else {
                // all 18 ring dwords: positions past outpos are not final and are rewritten
                // later; they stay below the records not yet read
#pragma unroll
                for (int j = 0; j < kRcRing / 4; j++) stage32[(base >> 2) + j] = ring32[j];
            }
        } else {
            const uint32_t m = (uint32_t)(n & 63);
#pragma unroll 1
            for (uint32_t k = 0; k < m; k++) c.step_exact(rec_at(cur, (int)k));
        }
#pragma unroll
        for (int j = 0; j < 32; j++) cur[j] = nxt[j];
    }
    if (sk == kRcSegs - 1 && a.flush) {
#pragma unroll 1
        for (int k = 0; k < 5; k++) c.shift_low();   // FlushData (:31-36)
    }
    seg[1] = c.outpos; seg[2] = c.lo; seg[3] = c.carry; seg[4] = c.cache; seg[5] = c.cache_size; seg[6] = c.range;
}

// the segments of a stream into the caller's output layout (one workgroup per stream):
// emitted bytes copied in parallel, then thread 0 adds each segment's unfinished digits
// into the next segment's first bytes, carries running toward the stream start
__global__ void __launch_bounds__(256) rc_merge_kernel(RcArgs a) {
    const uint32_t s = blockIdx.x;
    if (a.status[s] != LZMA_OK) return;
    const uint32_t* seg = a.seg + (size_t)s * kRcSegs * kRcSegWords;
    const uint64_t nall = a.rec_lens[s], seglen = rc_seglen(nall, a.sliced);
    uint64_t pos[kRcSegs + 1];
    pos[0] = 0;
    for (int k = 0; k < kRcSegs; k++) {
        const uint32_t* g = seg + k * kRcSegWords;
        pos[k + 1] = pos[k] + g[1] + g[5] - 1;
    }
    // an unflushed slice (the sliced encode): its output ends with the last non-empty
    // segment's emitted bytes; that segment's unfinished digits and end range are the
    // coder's state for the next slice (rc_seglen)
    const int last = (a.sliced && !a.flush) ? (seglen >= nall ? 0 : kRcSegs - 1) : kRcSegs - 1;
    const uint64_t total = pos[last] + seg[last * kRcSegWords + 1];
    if (a.sliced && !a.flush && threadIdx.x == 0) {
        const uint32_t* g = seg + last * kRcSegWords;
        uint32_t* es = a.end_state + (size_t)s * kRcStateWords;
        es[0] = g[6]; es[1] = g[2]; es[2] = g[3]; es[3] = g[4]; es[4] = g[5];
        if (last > 0 && g[1] < 5) a.status[s] = LZMA_E_INTERNAL;   // an earlier tail would reach its digits (rc_seglen)
    }
    const uint64_t cap = a.out_offs[s + 1] - a.out_offs[s];
    if (threadIdx.x == 0) a.out_lens[s] = total;
    if (total > cap) {
        if (threadIdx.x == 0) a.status[s] = LZMA_E_OVERFLOW;
        return;
    }
    uint8_t* dst = a.out + a.out_offs[s];
    for (int k = 0; k <= last; k++) {
        const uint8_t* src = (const uint8_t*)(a.recs + a.rec_offs[s] + rc_split(nall, seglen, k));
        const uint32_t len = seg[k * kRcSegWords + 1];
        const uint64_t end = k < last ? pos[k + 1] : total;   // the pending digits start as 0
        for (uint64_t j = threadIdx.x; j < end - pos[k]; j += blockDim.x) dst[pos[k] + j] = j < len ? src[j] : 0;
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    for (int k = 0; k < last; k++) {
        const uint32_t* g = seg + k * kRcSegWords;
        const uint32_t len = g[1], lo = g[2], cy = g[3], cache = g[4], cs = g[5];
        const uint64_t q0 = pos[k] + len;   // the cache digit
        // digits of the unfinished part, least significant first: low's 4 bytes, then the
        // pending group (cs - 1 x 0xFF, the cache) with the coder's carry at its last digit
        uint32_t carry = 0;
        for (int t = (int)cs + 3; t >= 0; t--) {
            const uint64_t q = q0 + (uint64_t)t;
            uint32_t d;
            if (t >= (int)cs) d = (lo >> (8 * (3 - (t - (int)cs)))) & 0xFFu;
            else d = t == 0 ? cache : 0xFFu;
            if (t == (int)cs - 1) d += cy;
            const uint32_t v = (uint32_t)dst[q] + d + carry;
            dst[q] = (uint8_t)v;
            carry = v >> 8;
        }
        for (uint64_t q = q0; carry && q > 0;) {   // rare: through earlier 0xFF digits
            q--;
            const uint32_t v = (uint32_t)dst[q] + carry;
            dst[q] = (uint8_t)v;
            carry = v >> 8;
        }
    }
}

int launch_rc(Ctx* ctx, const RcArgs& a, hipStream_t st) {
    if (a.nstreams <= 0) return LZMA_OK;
    {
        TimedLaunch tl(ctx, "enc_rc", st);
        hipLaunchKernelGGL(rc_range_kernel, dim3((a.nstreams + kRcLanes - 1) / kRcLanes), dim3(kRcLanes), 0, st, a);
        const int lanes = a.nstreams * kRcSegs;
        hipLaunchKernelGGL(rc_kernel, dim3((lanes + kRcLanes - 1) / kRcLanes), dim3(kRcLanes), 0, st, a);
        hipLaunchKernelGGL(rc_merge_kernel, dim3(a.nstreams), dim3(256), 0, st, a);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "rc launch: %s", hipGetErrorString(e));
    return LZMA_OK;
}

}  // namespace lzg
