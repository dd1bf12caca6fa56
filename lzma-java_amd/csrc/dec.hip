// dec.hip -- batched LZMA decoder: src/main/java/SevenZip/Compression/LZMA/
// Decoder.java (Code :205-301) with RangeDecoder.java and OutWindow.java, one
// wavefront (kWave = 64 lanes) per independent stream, one workgroup per
// stream (longest first).
//
// The DecodeBit chain is strictly serial, so it runs as wave-uniform scalar
// code; the probability models live in LDS. Memory round trips are kept off
// that chain:
//   * compressed input is staged through an LDS ring (kIbuf bytes, refilled
//     by all lanes at once), so RangeDecoder's byte reads are LDS reads;
//   * the most recent kWin output bytes live in an LDS window (OutWindow,
//     OutWindow.java:15-82); match copies and matched-literal bytes read it,
//     with all lanes copying (an overlapping copy repeats the d-byte period:
//     out[now + k] = out[now - d + k % d]);
//   * the window is flushed to HBM kFlush bytes at a time (coalesced); a
//     distance beyond half the window reads the flushed bytes in HBM.
#include "lzma_common.h"
#include "runtime.h"

namespace lzg {

constexpr int kDecLitLdsMaxBits = 3;
constexpr uint32_t kIbuf = 128;     // input staging ring
constexpr uint32_t kWin = 1024;     // output window in LDS (power of two)
constexpr uint32_t kFlush = 128;    // window -> HBM flush granule
constexpr uint32_t kNear = kWin / 2;   // distances <= kNear read the LDS window
static_assert(kFlush + kMatchMaxLen + 64 <= kNear, "window too small for the flush lag");

#define DFI __device__ __forceinline__
#define LANE_FENCE() asm volatile("" ::: "memory")

DFI uint64_t dec_uni64(uint64_t v) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}

// LIT_LDS: literal coders in LDS (lc + lp <= 3) or HBM. A compile-time choice,
// so every pointer has a known address space (a generic pointer would make the
// compiler treat each loaded model as per-lane and the whole decode as divergent).
// PBS: posState stride of the probability layout (ProbLayout, lzma_common.h).
template <bool LIT_LDS, int PBS>
struct Dec {
    using PL = ProbLayout<PBS>;
    uint32_t lane;
    uint16_t* probs;
    uint16_t* lit;
    uint8_t* ibuf;                // [kIbuf]
    uint8_t* win;                 // [kWin]
    uint32_t lc, lp, pb, ps_mask, dict_check;
    const uint8_t* in;
    uint64_t n_in, ipos, ibase;
    uint8_t* out;
    __amdgpu_buffer_rsrc_t outb;  // the stream's output as a buffer (far reads; never merged with LDS reads)
    uint64_t cap, flushed;
    uint32_t range, code;

    // ---- input (InputStream.read(): -1 past the end)
    DFI void refill(uint64_t base) {
        ibase = base;
        for (uint32_t k0 = 0; k0 < kIbuf; k0 += kWave) {   // uniform trip count
            const uint32_t k = k0 + lane;
            const uint64_t q = base + k;
            ibuf[k] = q < n_in ? in[q] : 0;
        }
        LANE_FENCE();
    }
    DFI uint32_t rd_byte() {
        if (ipos >= n_in) return 0xFFFFFFFFu;
        if (ipos - ibase >= kIbuf) refill(ipos);
        return (uint32_t)ibuf[(uint32_t)(ipos++ - ibase)];
    }
    // ---- output window
    DFI void flush_to(uint64_t upto) {   // write [flushed, upto) to HBM (upto <= now, within the window)
        LANE_FENCE();
        for (uint64_t k0 = flushed; k0 < upto; k0 += kWave) {   // uniform trip count
            const uint64_t k = k0 + lane;
            if (k < upto) out[k] = win[(uint32_t)k & (kWin - 1)];
        }
        flushed = upto;
        LANE_FENCE();
    }
    DFI void maybe_flush(uint64_t now) {
        if (now - flushed >= kFlush) flush_to(now & ~(uint64_t)(kFlush - 1));
    }
    DFI uint32_t byte_back(uint64_t now, uint32_t d1) {   // out[now - d1], 1 <= d1 <= now
        if (d1 <= kNear) return win[(uint32_t)(now - d1) & (kWin - 1)];
        // flushed long ago (d1 > kNear > flush lag); streams < 2 GiB: 32-bit offsets
        return __builtin_amdgcn_raw_buffer_load_b8(outb, (uint32_t)(now - d1), 0, 0);
    }
    DFI void put(uint64_t now, uint32_t b) {
        if (lane == 0) win[(uint32_t)now & (kWin - 1)] = (uint8_t)b;
        LANE_FENCE();
    }

    // ---- range decoder
    DFI uint32_t bit(uint16_t* p, uint32_t idx) {   // RangeDecoder.DecodeBit (RangeDecoder.java:43-64)
        uint32_t prob = p[idx];
        uint32_t bound = (range >> 11) * prob;
        uint32_t r;
        if (code < bound) {
            range = bound;
            p[idx] = (uint16_t)(prob + ((kBitModelTotal - prob) >> kNumMoveBits));
            r = 0;
        } else {
            range -= bound;
            code -= bound;
            p[idx] = (uint16_t)(prob - (prob >> kNumMoveBits));
            r = 1;
        }
        if ((range & kTopMask) == 0) { code = (code << 8) | rd_byte(); range <<= 8; }
        return r;
    }
    DFI uint32_t direct(int nbits) {   // RangeDecoder.DecodeDirectBits (RangeDecoder.java:27-41)
        uint32_t result = 0;
        for (int i = nbits; i != 0; i--) {
            range >>= 1;
            uint32_t t = (code - range) >> 31;
            code -= range & (t - 1);
            result = (result << 1) | (1 - t);
            if ((range & kTopMask) == 0) { code = (code << 8) | rd_byte(); range <<= 8; }
        }
        return result;
    }
    DFI uint32_t bt_dec(uint16_t* p, int nbits) {   // BitTreeDecoder.Decode (BitTreeDecoder.java:19-25)
        uint32_t m = 1;
        for (int b = nbits; b != 0; b--) m = (m << 1) + bit(p, m);
        return m - (1u << nbits);
    }
    DFI uint32_t bt_rev_dec(uint16_t* p, int nbits) {   // BitTreeDecoder.ReverseDecode (:27-37)
        uint32_t m = 1, sym = 0;
        for (int b = 0; b < nbits; b++) { uint32_t x = bit(p, m); m <<= 1; m += x; sym |= x << b; }
        return sym;
    }
    DFI uint32_t len_dec(uint16_t* L, uint32_t ps) {   // Decoder.LenDecoder.Decode (Decoder.java:48-59)
        if (bit(L, LEN_CHOICE) == 0) return bt_dec(L + PL::LOW + ps * 8, 3);
        uint32_t sym = kNumLowLenSymbols;
        if (bit(L, LEN_CHOICE + 1) == 0) sym += bt_dec(L + PL::MID + ps * 8, 3);
        else sym += kNumMidLenSymbols + bt_dec(L + PL::HIGH, 8);
        return sym;
    }
    // OutWindow.CopyBlock (OutWindow.java:53-67) of len bytes at distance d1,
    // byte-serial semantics: an overlapping copy repeats the d1-byte period.
    DFI void copy(uint64_t now, uint32_t d1, uint32_t len) {
        LANE_FENCE();
        for (uint32_t k0 = 0; k0 < len; k0 += kWave) {
            const uint32_t k = k0 + lane;
            if (k < len) {
                // source = now - d1 + (k mod d1): always before `now`, so lanes never
                // read a byte this copy writes (and kNear + 273 < kWin: no ring alias)
                const uint32_t r = k % d1;
                win[(uint32_t)(now + k) & (kWin - 1)] = (uint8_t)byte_back(now, d1 - r);
            }
        }
        LANE_FENCE();
    }

    // returns LZMA_OK / LZMA_E_DATA / LZMA_E_OVERFLOW; *now_out = bytes written
    DFI int run(int64_t out_size, uint64_t* now_out) {
        const uint32_t nlit = 0x300u << (lc + lp);
        for (uint32_t i0 = 0; i0 < (uint32_t)PL::COUNT; i0 += kWave)
            if (i0 + lane < (uint32_t)PL::COUNT) probs[i0 + lane] = kBitModelTotal >> 1;
        for (uint32_t i0 = 0; i0 < nlit; i0 += kWave)
            if (i0 + lane < nlit) lit[i0 + lane] = kBitModelTotal >> 1;
        LANE_FENCE();
        ipos = 0;
        ibase = 0;
        refill(0);
        flushed = 0;
        code = 0;
        range = 0xFFFFFFFFu;
        for (int i = 0; i < 5; i++) code = (code << 8) | rd_byte();   // RangeDecoder.Init
        uint32_t state = 0, rep0 = 0, rep1 = 0, rep2 = 0, rep3 = 0;
        uint64_t now = 0;
        uint32_t prev = 0;
        int rc = LZMA_OK;
        while (out_size < 0 || (int64_t)now < out_size) {
            const uint32_t ps = (uint32_t)now & ps_mask;
            if (bit(probs + PL::IS_MATCH, (state << PBS) + ps) == 0) {
                uint16_t* sub = lit + (size_t)((((uint32_t)now & ((1u << lp) - 1)) << lc) + (prev >> (8 - lc))) * 0x300;
                uint32_t sym = 1;
                if (st_is_char(state)) {
                    do { sym = (sym << 1) | bit(sub, sym); } while (sym < 0x100);
                } else {   // LiteralDecoder.Decoder2.DecodeWithMatchByte (Decoder.java:80-102)
                    uint32_t mb = byte_back(now, rep0 + 1);
                    do {
                        uint32_t mbit = (mb >> 7) & 1;
                        mb <<= 1;
                        uint32_t b = bit(sub, ((1 + mbit) << 8) + sym);
                        sym = (sym << 1) | b;
                        if (mbit != b) {
                            while (sym < 0x100) sym = (sym << 1) | bit(sub, sym);
                            break;
                        }
                    } while (sym < 0x100);
                }
                prev = sym & 0xFF;
                if (now >= cap) { rc = LZMA_E_OVERFLOW; break; }
                put(now, prev);
                now++;
                state = st_lit(state);
            } else {
                uint32_t len;
                if (bit(probs + PL::IS_REP, state) == 1) {
                    len = 0;
                    if (bit(probs + PL::G0, state) == 0) {
                        if (bit(probs + PL::R0L, (state << PBS) + ps) == 0) { state = st_short(state); len = 1; }
                    } else {
                        uint32_t dist;
                        if (bit(probs + PL::G1, state) == 0) dist = rep1;
                        else {
                            if (bit(probs + PL::G2, state) == 0) dist = rep2;
                            else { dist = rep3; rep3 = rep2; }
                            rep2 = rep1;
                        }
                        rep1 = rep0;
                        rep0 = dist;
                    }
                    if (len == 0) { len = len_dec(probs + PL::RLEN, ps) + kMatchMinLen; state = st_long(state); }
                } else {
                    rep3 = rep2; rep2 = rep1; rep1 = rep0;
                    len = kMatchMinLen + len_dec(probs + PL::LEN, ps);
                    state = st_match(state);
                    uint32_t slot = bt_dec(probs + PL::PSLOT + (len_to_pos_state(len) << 6), kNumPosSlotBits);
                    if (slot >= (uint32_t)kStartPosModelIndex) {
                        uint32_t ndb = (slot >> 1) - 1;
                        rep0 = (2 | (slot & 1)) << ndb;
                        if (slot < (uint32_t)kEndPosModelIndex) {
                            rep0 += bt_rev_dec(probs + PL::PENC + (int32_t)(rep0 - slot - 1), (int)ndb);
                        } else {
                            rep0 += direct((int)(ndb - kNumAlignBits)) << kNumAlignBits;
                            rep0 += bt_rev_dec(probs + PL::ALIGN, kNumAlignBits);
                            if ((int32_t)rep0 < 0) {
                                if (rep0 == 0xFFFFFFFFu) break;   // end marker
                                rc = LZMA_E_DATA;
                                break;
                            }
                        }
                    } else {
                        rep0 = slot;
                    }
                }
                if ((uint64_t)rep0 >= now || rep0 >= dict_check) { rc = LZMA_E_DATA; break; }
                const uint32_t d1 = rep0 + 1;
                if (now + len > cap) {   // copy what fits, then report (no bytes past the capacity)
                    const uint32_t fit = (uint32_t)(cap - now);
                    copy(now, d1, fit);
                    now = cap;
                    rc = LZMA_E_OVERFLOW;
                    break;
                }
                copy(now, d1, len);
                now += len;
                prev = win[(uint32_t)(now - 1) & (kWin - 1)];
            }
            maybe_flush(now);
        }
        flush_to(now);
        *now_out = now;
        return rc;
    }
};

template <bool LIT_LDS, int PBS>
__global__ void __launch_bounds__(kWave) dec_kernel(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Dec<LIT_LDS, PBS> d;
    d.lane = threadIdx.x;
    d.lc = a.lc; d.lp = a.lp; d.pb = a.pb; d.ps_mask = (1u << a.pb) - 1; d.dict_check = a.dict_check;
    size_t off = 0;
    auto take = [&](size_t bytes) { uint8_t* p = smem + off; off += (bytes + 15) & ~(size_t)15; return p; };
    d.probs = (uint16_t*)take((size_t)ProbLayout<PBS>::COUNT * 2);
    d.ibuf = take(kIbuf);
    d.win = take(kWin);
    if (LIT_LDS) d.lit = (uint16_t*)take(((size_t)0x300 << (a.lc + a.lp)) * 2);
    else d.lit = (uint16_t*)(a.scratch + (size_t)blockIdx.x * a.scratch_stride);
    // one workgroup per stream; per-stream values are wave-uniform (readfirstlane keeps them scalar)
    const int s = __builtin_amdgcn_readfirstlane((int)a.order[blockIdx.x]);
    const uint64_t i0 = dec_uni64(a.in_offs[s]), o0 = dec_uni64(a.out_offs[s]);
    d.in = a.in + i0;
    d.n_in = dec_uni64(a.in_offs[s + 1]) - i0;
    d.out = a.out + o0;
    d.cap = dec_uni64(a.out_offs[s + 1]) - o0;
    d.outb = __builtin_amdgcn_make_buffer_rsrc(d.out, 0, d.cap > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d.cap, 0x00020000);
    const int64_t out_size = (int64_t)dec_uni64((uint64_t)a.out_sizes[s]);
    uint64_t now = 0;
    int rc = d.run(out_size, &now);
    if (d.lane == 0) { a.out_lens[s] = now; a.status[s] = rc; }
}

size_t dec_scratch_per_block(uint32_t lc, uint32_t lp) { return ((size_t)0x300 << (lc + lp)) * 2 + 256; }

static size_t dec_lds_bytes(uint32_t lc, uint32_t lp, uint32_t pb, uint32_t lit_in_lds) {
    auto r = [](size_t b) { return (b + 15) & ~(size_t)15; };
    size_t lds = r((size_t)prob_count(pb) * 2) + r(kIbuf) + r(kWin);
    if (lit_in_lds) lds += r(((size_t)0x300 << (lc + lp)) * 2);
    return lds;
}

int dec_grid(uint32_t, uint32_t, uint32_t, int nstreams) { return nstreams; }   // one workgroup per stream

template <bool LIT, int PBS>
static void launch_dec(const DecArgs& a, int grid, size_t lds, hipStream_t st) {
    if (lds > 64 * 1024) hipFuncSetAttribute((const void*)dec_kernel<LIT, PBS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((dec_kernel<LIT, PBS>), dim3(grid), dim3(kWave), lds, st, a);
}

int launch_decoder(Ctx* ctx, const DecArgs& a, int grid, hipStream_t st) {
    size_t lds = dec_lds_bytes(a.lc, a.lp, a.pb, a.lit_in_lds);
    TimedLaunch tl(ctx, "dec_stream", st);
    if (a.lit_in_lds) {
        if (a.pb <= 2) launch_dec<true, 2>(a, grid, lds, st); else launch_dec<true, 4>(a, grid, lds, st);
    } else {
        if (a.pb <= 2) launch_dec<false, 2>(a, grid, lds, st); else launch_dec<false, 4>(a, grid, lds, st);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "dec launch: %s", hipGetErrorString(e));
    return LZMA_OK;
}

}  // namespace lzg
