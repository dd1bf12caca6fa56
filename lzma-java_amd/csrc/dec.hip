// dec.hip -- batched LZMA decoder: src/main/java/SevenZip/Compression/LZMA/
// Decoder.java (Code :205-301) with RangeDecoder.java and OutWindow.java, one
// wavefront (kWave = 64 lanes) per independent stream pulled from a work queue.
//
// The DecodeBit chain is strictly serial, so it runs as wave-uniform code;
// the probability models live in LDS. The output buffer in HBM is the window
// (OutWindow's ring is unobservable when the whole output is resident), and
// long match copies (OutWindow.CopyBlock, OutWindow.java:53-67) use all
// lanes when the source lies wholly before the destination.
#include "lzma_common.h"
#include "runtime.h"

namespace lzg {

constexpr int kDecLitLdsMaxBits = 3;

#define WSYNC() __syncthreads()

struct Dec {
    int lane;
    uint16_t* probs;
    uint16_t* lit;
    uint32_t lc, lp, pb, ps_mask, dict_check;
    const uint8_t* in;
    uint64_t n_in, ipos;
    uint8_t* out;
    uint64_t cap;
    uint32_t range, code;

    __device__ uint32_t rd_byte() {   // InputStream.read(): -1 past the end
        return ipos < n_in ? (uint32_t)in[ipos++] : 0xFFFFFFFFu;
    }
    __device__ uint32_t bit(uint16_t* p, uint32_t idx) {   // RangeDecoder.DecodeBit (RangeDecoder.java:43-64)
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
    __device__ uint32_t direct(int nbits) {   // RangeDecoder.DecodeDirectBits (RangeDecoder.java:27-41)
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
    __device__ uint32_t bt_dec(uint16_t* p, int nbits) {   // BitTreeDecoder.Decode
        uint32_t m = 1;
        for (int b = nbits; b != 0; b--) m = (m << 1) + bit(p, m);
        return m - (1u << nbits);
    }
    __device__ uint32_t bt_rev_dec(uint16_t* p, int nbits) {   // BitTreeDecoder.ReverseDecode / Decoder.ReverseDecode
        uint32_t m = 1, sym = 0;
        for (int b = 0; b < nbits; b++) { uint32_t x = bit(p, m); m <<= 1; m += x; sym |= x << b; }
        return sym;
    }
    __device__ uint32_t len_dec(uint16_t* L, uint32_t ps) {   // Decoder.LenDecoder.Decode (Decoder.java:48-59)
        if (bit(L, LEN_CHOICE) == 0) return bt_dec(L + LEN_LOW + ps * 8, 3);
        uint32_t sym = kNumLowLenSymbols;
        if (bit(L, LEN_CHOICE + 1) == 0) sym += bt_dec(L + LEN_MID + ps * 8, 3);
        else sym += kNumMidLenSymbols + bt_dec(L + LEN_HIGH, 8);
        return sym;
    }

    // returns LZMA_OK / LZMA_E_DATA / LZMA_E_OVERFLOW; *now = bytes written
    __device__ int run(int64_t out_size, uint64_t* now_out) {
        const uint32_t nlit = 0x300u << (lc + lp);
        for (uint32_t i = lane; i < (uint32_t)P_FIXED_COUNT; i += kWave) probs[i] = kBitModelTotal >> 1;
        for (uint32_t i = lane; i < nlit; i += kWave) lit[i] = kBitModelTotal >> 1;
        WSYNC();
        ipos = 0;
        code = 0;
        range = 0xFFFFFFFFu;
        for (int i = 0; i < 5; i++) code = (code << 8) | rd_byte();   // RangeDecoder.Init
        uint32_t state = 0, rep0 = 0, rep1 = 0, rep2 = 0, rep3 = 0;
        uint64_t now = 0;
        uint32_t prev = 0;
        int rc = LZMA_OK;
        while (out_size < 0 || (int64_t)now < out_size) {
            uint32_t ps = (uint32_t)now & ps_mask;
            if (bit(probs + P_IS_MATCH, (state << 4) + ps) == 0) {
                uint16_t* sub = lit + (size_t)((((uint32_t)now & ((1u << lp) - 1)) << lc) + (prev >> (8 - lc))) * 0x300;
                uint32_t sym = 1;
                if (st_is_char(state)) {
                    do { sym = (sym << 1) | bit(sub, sym); } while (sym < 0x100);
                } else {
                    uint32_t mb = out[now - rep0 - 1];
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
                out[now] = (uint8_t)prev;
                now++;
                state = st_lit(state);
            } else {
                uint32_t len;
                if (bit(probs + P_IS_REP, state) == 1) {
                    len = 0;
                    if (bit(probs + P_IS_REP_G0, state) == 0) {
                        if (bit(probs + P_IS_REP0_LONG, (state << 4) + ps) == 0) { state = st_short(state); len = 1; }
                    } else {
                        uint32_t dist;
                        if (bit(probs + P_IS_REP_G1, state) == 0) dist = rep1;
                        else {
                            if (bit(probs + P_IS_REP_G2, state) == 0) dist = rep2;
                            else { dist = rep3; rep3 = rep2; }
                            rep2 = rep1;
                        }
                        rep1 = rep0;
                        rep0 = dist;
                    }
                    if (len == 0) { len = len_dec(probs + P_REP_LEN, ps) + kMatchMinLen; state = st_long(state); }
                } else {
                    rep3 = rep2; rep2 = rep1; rep1 = rep0;
                    len = kMatchMinLen + len_dec(probs + P_LEN, ps);
                    state = st_match(state);
                    uint32_t slot = bt_dec(probs + P_POS_SLOT + (len_to_pos_state(len) << 6), kNumPosSlotBits);
                    if (slot >= (uint32_t)kStartPosModelIndex) {
                        uint32_t ndb = (slot >> 1) - 1;
                        rep0 = (2 | (slot & 1)) << ndb;
                        if (slot < (uint32_t)kEndPosModelIndex) {
                            rep0 += bt_rev_dec(probs + P_POS_ENC + (int32_t)(rep0 - slot - 1), (int)ndb);
                        } else {
                            rep0 += direct((int)(ndb - kNumAlignBits)) << kNumAlignBits;
                            rep0 += bt_rev_dec(probs + P_ALIGN, kNumAlignBits);
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
                // OutWindow.CopyBlock: byte-serial semantics (overlapping copies repeat the pattern)
                uint64_t d1 = (uint64_t)rep0 + 1;
                if (now + len > cap) {   // copy what fits, then report (no bytes past the capacity)
                    for (uint64_t k = 0; now + k < cap; k++) out[now + k] = out[now + k - d1];
                    now = cap;
                    rc = LZMA_E_OVERFLOW;
                    break;
                }
                if (d1 >= len && len >= 32) {   // source fully written before the copy starts
                    WSYNC();
                    for (uint32_t k = lane; k < len; k += kWave) out[now + k] = out[now + k - d1];
                    WSYNC();
                } else {
                    for (uint32_t k = 0; k < len; k++) out[now + k] = out[now + k - d1];
                }
                now += len;
                prev = out[now - 1];
            }
        }
        *now_out = now;
        return rc;
    }
};

__global__ void __launch_bounds__(kWave) dec_kernel(DecArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Dec d;
    d.lane = threadIdx.x;
    d.lc = a.lc; d.lp = a.lp; d.pb = a.pb; d.ps_mask = (1u << a.pb) - 1; d.dict_check = a.dict_check;
    d.probs = (uint16_t*)smem;
    size_t off = ((size_t)P_FIXED_COUNT * 2 + 15) & ~(size_t)15;
    if (a.lit_in_lds) d.lit = (uint16_t*)(smem + off);
    else d.lit = (uint16_t*)(a.scratch + blockIdx.x * a.scratch_stride);
    for (;;) {
        int idx = 0;
        if (d.lane == 0) idx = (int)atomicAdd(a.next, 1u);
        idx = __shfl(idx, 0);
        if (idx >= a.nstreams) break;
        int s = (int)a.order[idx];
        d.in = a.in + a.in_offs[s];
        d.n_in = a.in_offs[s + 1] - a.in_offs[s];
        d.out = a.out + a.out_offs[s];
        d.cap = a.out_offs[s + 1] - a.out_offs[s];
        uint64_t now = 0;
        int rc = d.run(a.out_sizes[s], &now);
        if (d.lane == 0) { a.out_lens[s] = now; a.status[s] = rc; }
        WSYNC();
    }
}

size_t dec_scratch_per_block(uint32_t lc, uint32_t lp) { return ((size_t)0x300 << (lc + lp)) * 2 + 256; }

static size_t dec_lds_bytes(uint32_t lc, uint32_t lp, uint32_t lit_in_lds) {
    size_t lds = ((size_t)P_FIXED_COUNT * 2 + 15) & ~(size_t)15;
    if (lit_in_lds) lds += ((size_t)0x300 << (lc + lp)) * 2;
    return lds;
}

int dec_grid(uint32_t lc, uint32_t lp, uint32_t lit_in_lds, int nstreams) {
    size_t lds = dec_lds_bytes(lc, lp, lit_in_lds);
    int dev = 0;
    hipGetDevice(&dev);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
    int per_cu = (int)((160 * 1024) / (lds + 256));
    if (per_cu > 16) per_cu = 16;
    if (per_cu < 1) per_cu = 1;
    int grid = cus * per_cu;
    if (grid > nstreams) grid = nstreams;
    if (grid < 1) grid = 1;
    return grid;
}

int launch_decoder(Ctx* ctx, const DecArgs& a, int grid, hipStream_t st) {
    size_t lds = dec_lds_bytes(a.lc, a.lp, a.lit_in_lds);
    TimedLaunch tl(ctx, "dec_stream", st);
    hipLaunchKernelGGL(dec_kernel, dim3(grid), dim3(kWave), lds, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "dec launch: %s", hipGetErrorString(e));
    return LZMA_OK;
}

}  // namespace lzg
