// dec.hip -- batched LZMA decoder: src/main/java/SevenZip/Compression/LZMA/
// Decoder.java (Code :205-301) with RangeDecoder.java, BitTreeDecoder.java and
// OutWindow.java, one wavefront (kWave = 64 lanes) per independent stream,
// one workgroup per stream (longest first).
//
// The DecodeBit chain is strictly serial, so it runs as wave-uniform scalar
// code. What the lanes do is keep memory round trips off that chain:
//   * bit trees are prefetched whole: before a tree is walked, every lane
//     loads one or two of its nodes (one LDS or HBM round trip for the whole
//     tree instead of one per bit); the walk reads the node probabilities out
//     of the lanes (readlane) and writes each adapted probability back as it
//     goes (the nodes along one path are distinct, so the prefetched values
//     stay exact for the rest of the walk);
//   * the literal coders (0x300 << (lc + lp) probabilities) live in a
//     per-stream HBM area, except (LITP: lc + lp <= 3 and at most 8 streams per CU)
//     their plain 256-node trees, which take 4 KiB of LDS: a literal outside matched
//     mode then touches no HBM (at 16 streams per CU the LDS is left to the match
//     finder's sorts a pipelined caller runs beside the decode); a literal's whole coder tree (plus
//     the 8 matched-mode nodes along the match byte) is fetched in one round trip,
//     issued before the isMatch decision so it overlaps with it;
//   * compressed input is staged through an LDS ring (kIbuf bytes, refilled
//     by all lanes at once);
//   * the most recent kWin output bytes live in an LDS window (OutWindow,
//     OutWindow.java:15-82); match copies and matched-literal bytes read it
//     with all lanes copying (an overlapping copy repeats the d-byte period:
//     out[now + k] = out[now - d + k % d]); distances beyond half the window
//     read the flushed bytes in HBM;
//   * the window is flushed to HBM kFlush bytes at a time (coalesced).
#include "lzma_common.h"
#include "runtime.h"

namespace lzg {

#ifndef LZG_DEC_FLUSH_NT
#define LZG_DEC_FLUSH_NT 1   // the window's flush to HBM as non-temporal stores (A/B: 0 = cached stores)
#endif

constexpr uint32_t kIbuf = 256;     // input staging ring
constexpr uint32_t kWin = 1024;     // output window in LDS (power of two)
constexpr uint32_t kFlush = 128;    // window -> HBM flush granule
constexpr uint32_t kNear = kWin / 2;   // distances <= kNear read the LDS window
static_assert(kFlush + kMatchMaxLen + 64 <= kNear, "window too small for the flush lag");
constexpr int kVS = (64 + kWave - 1) / kWave;   // per-lane slots of a 64-entry lane vector (1 on hardware)

#define DFI __device__ __forceinline__
#define LANE_FENCE() asm volatile("" ::: "memory")

DFI uint64_t dec_uni64(uint64_t v) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}
// element j (wave-uniform, < 64) of a lane vector: lane j % kWave, slot j / kWave
DFI uint32_t vget(const uint32_t (&v)[kVS], uint32_t j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v[j / kWave], (int)(j % kWave));
}

// PBS: posState stride of the probability layout (ProbLayout, lzma_common.h).
// FairPrio rows of the decoder's waves (lzma_common.h)
__device__ uint32_t g_dec_sched[kSchedRows * kSchedCols];

constexpr uint32_t kDecLitpBits = 3;   // LITP: lc + lp <= 3 (at most 8 plain trees of 256 nodes in LDS)

template <int PBS, bool LITP>
struct Dec {
    using PL = ProbLayout<PBS>;
    uint32_t lane;
    uint16_t* probs;              // LDS: fixed models
    uint16_t* lit;                // HBM: literal coders of this stream
    uint16_t* litp;               // LITP: LDS, the plain trees (nodes 0x000-0x0FF of each coder), 256 per coder
    uint8_t* ibuf;                // LDS [kIbuf]
    uint8_t* win;                 // LDS [kWin]
    uint32_t lc, lp, pb, ps_mask, dict_check;
    const uint8_t* in;
    // streams < 4 GiB in and out (the host clamps the capacity): 32-bit positions keep the
    // scalar chain free of 64-bit compares
    uint32_t n_in, ipos, ibase, ilim;   // ilim = min(ibase + kIbuf, n_in): the fast-path bound
    uint8_t* out;
    __amdgpu_buffer_rsrc_t outb;  // the stream's output as a buffer (far reads; never merged with LDS reads)
    uint32_t cap, flushed;
    uint32_t range, code;

    // ---- input (InputStream.read(): -1 past the end)
    DFI void refill(uint32_t base) {
        ibase = base;
        ilim = n_in - base < kIbuf ? n_in : base + kIbuf;
        for (uint32_t k0 = 0; k0 < kIbuf; k0 += kWave) {   // uniform trip count
            const uint32_t k = k0 + lane;
            const uint32_t q = base + k;
            ibuf[k] = q < n_in ? __builtin_nontemporal_load(in + q) : 0;   // streamed once
        }
        LANE_FENCE();
    }
    DFI uint32_t rd_byte() {
        if (ipos >= ilim) {
            if (ipos >= n_in) return 0xFFFFFFFFu;
            refill(ipos);
        }
        return (uint32_t)ibuf[ipos++ - ibase];
    }
    // ---- output window
    DFI void flush_to(uint32_t upto) {   // write [flushed, upto) to HBM (upto <= now, within the window)
        LANE_FENCE();
        for (uint32_t k0 = flushed; k0 < upto; k0 += kWave) {   // uniform trip count
            const uint32_t k = k0 + lane;
            if (k < upto) {
                if (LZG_DEC_FLUSH_NT) __builtin_nontemporal_store(win[k & (kWin - 1)], out + k);
                else out[k] = win[k & (kWin - 1)];   // cached: a far match reads its source back from L2 / MALL
            }
        }
        flushed = upto;
        LANE_FENCE();
    }
    DFI void maybe_flush(uint32_t now) {
        if (now - flushed >= kFlush) flush_to(now & ~(kFlush - 1));
    }
    DFI uint32_t byte_back(uint32_t now, uint32_t d1) {   // out[now - d1], 1 <= d1 <= now
        if (d1 <= kNear) return win[(now - d1) & (kWin - 1)];
        // flushed long ago (d1 > kNear > flush lag)
        return __builtin_amdgcn_raw_buffer_load_b8(outb, now - d1, 0, 0);
    }
    DFI void put(uint32_t now, uint32_t b) {   // every lane stores the same byte: no exec-mask juggling
        win[now & (kWin - 1)] = (uint8_t)b;
        LANE_FENCE();
    }

    // ---- range decoder
    // RangeDecoder.DecodeBit (RangeDecoder.java:43-64) on a probability already
    // in a register; *np = the adapted probability
    // (branch-free selects: the scalar unit is the decoder's bottleneck)
    // The adapted probability only feeds a store, so it is computed on the vector
    // unit (vgpr(): a v_mov the compiler must treat as per-lane), off the scalar chain.
    static DFI uint32_t vgpr(uint32_t x) {
#if LZG_WAVE == 64
        uint32_t y;
        asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
        return y;
#else
        return x;
#endif
    }
    DFI uint32_t dbit(uint32_t prob, uint32_t* np) {
        const uint32_t bound = (range >> 11) * prob;
        const bool one = code >= bound;
        range = one ? range - bound : bound;
        code = one ? code - bound : code;
        const uint32_t pv = vgpr(prob), m = 0u - vgpr(one ? 1u : 0u);   // a lane mask, not a branch
        const uint32_t up = pv + ((kBitModelTotal - pv) >> kNumMoveBits), dn = pv - (pv >> kNumMoveBits);
        *np = up ^ ((up ^ dn) & m);
        if (range < (1u << 24)) { code = (code << 8) | rd_byte(); range <<= 8; }
        return one ? 1u : 0u;
    }
    DFI uint32_t bit(uint16_t* p, uint32_t idx) {   // one decision against an LDS model
        uint32_t np;
        const uint32_t r = dbit(p[idx], &np);
        p[idx] = (uint16_t)np;
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
    // ---- prefetched trees (LDS): node m (< 64) of p in lane m
    DFI void fetch64(const uint16_t* p, uint32_t n, uint32_t (&v)[kVS]) const {
#pragma unroll
        for (int s = 0; s < kVS; s++) {
            const uint32_t m = (uint32_t)(s * kWave) + lane;
            v[s] = m < n ? (uint32_t)p[m] : 0u;
        }
    }
    // BitTreeDecoder.Decode (BitTreeDecoder.java:19-25) over a prefetched tree (nbits <= 6)
    DFI uint32_t bt_dec(uint16_t* p, const uint32_t (&v)[kVS], int nbits) {
        uint32_t m = 1;
        for (int b = nbits; b != 0; b--) {
            uint32_t np;
            const uint32_t x = dbit(vget(v, m), &np);
            p[m] = (uint16_t)np;
            m = (m << 1) + x;
        }
        return m - (1u << nbits);
    }
    // BitTreeDecoder.ReverseDecode (:27-37) over a prefetched tree (nbits <= 5)
    DFI uint32_t bt_rev_dec(uint16_t* p, const uint32_t (&v)[kVS], int nbits) {
        uint32_t m = 1, sym = 0;
        for (int b = 0; b < nbits; b++) {
            uint32_t np;
            const uint32_t x = dbit(vget(v, m), &np);
            p[m] = (uint16_t)np;
            m = (m << 1) + x;
            sym |= x << b;
        }
        return sym;
    }
    // 256-node tree p[0..255] as four lane vectors: node m in lane m % 64 of vector m / 64,
    // so a walk's node read is one readlane with the node index (no half-word select)
    struct T256 { uint32_t v[4][kVS]; };
    template <typename P>
    DFI void fetch256(const P* p, T256& t) const {
#pragma unroll
        for (int k = 0; k < 4; k++)
#pragma unroll
            for (int s = 0; s < kVS; s++) t.v[k][s] = (uint32_t)p[64 * k + s * kWave + lane];
    }
    // node m of tree level `level` (m in [2^level, 2^(level+1)))
    DFI static uint32_t node256(const T256& t, uint32_t m, int level) {
        if (level <= 5) return vget(t.v[0], m);
        if (level == 6) return vget(t.v[1], m & 63u);
        return (m & 64u) ? vget(t.v[3], m & 63u) : vget(t.v[2], m & 63u);
    }
    // Decoder.LenDecoder.Decode (Decoder.java:48-59) over prefetched nodes:
    // lv lanes 0-7 low[ps], 8-15 mid[ps], 16-17 the two choices; lo/hi the high tree
    DFI void fetch_len(const uint16_t* L, uint32_t ps, uint32_t (&lv)[kVS], T256& ht) const {
#pragma unroll
        for (int s = 0; s < kVS; s++) {
            const uint32_t m = (uint32_t)(s * kWave) + lane;
            uint32_t v = 0;
            if (m < 8) v = L[PL::LOW + ps * 8 + m];
            else if (m < 16) v = L[PL::MID + ps * 8 + m - 8];
            else if (m < 18) v = L[LEN_CHOICE + m - 16];
            lv[s] = v;
        }
        fetch256(L + PL::HIGH, ht);
    }
    DFI uint32_t len_dec(uint16_t* L, uint32_t ps, const uint32_t (&lv)[kVS], const T256& ht) {
        uint32_t np;
        uint32_t x = dbit(vget(lv, 16), &np);
        L[LEN_CHOICE] = (uint16_t)np;
        uint32_t base, off, nb, sym0;
        if (x == 0) { base = PL::LOW + ps * 8; off = 0; nb = 3; sym0 = 0; }
        else {
            x = dbit(vget(lv, 17), &np);
            L[LEN_CHOICE + 1] = (uint16_t)np;
            if (x == 0) { base = PL::MID + ps * 8; off = 8; nb = 3; sym0 = kNumLowLenSymbols; }
            else { base = PL::HIGH; off = 0; nb = 8; sym0 = kNumLowLenSymbols + kNumMidLenSymbols; }
        }
        uint32_t m = 1;
        if (nb == 3) {   // unrolled walks: static trip counts and lane-vector choices
#pragma unroll
            for (int b = 0; b < 3; b++) {
                x = dbit(vget(lv, off + m), &np);
                L[base + m] = (uint16_t)np;
                m = (m << 1) + x;
            }
            return sym0 + m - 8u;
        }
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint32_t prob = node256(ht, m, b);
            x = dbit(prob, &np);
            L[base + m] = (uint16_t)np;
            m = (m << 1) + x;
        }
        return sym0 + m - 256u;
    }
    // OutWindow.CopyBlock (OutWindow.java:53-67) of len bytes at distance d1,
    // byte-serial semantics: an overlapping copy repeats the d1-byte period.
    // Returns the byte one past the copy, out[now + len - d1]: the match byte of a literal
    // that follows (Decoder.java:85, GetByte(rep0)), fetched in the copy's own round trip.
    DFI uint32_t copy(uint32_t now, uint32_t d1, uint32_t len) {
        LANE_FENCE();
        uint32_t next = 0;
        for (uint32_t k0 = 0; k0 <= len; k0 += kWave) {
            const uint32_t k = k0 + lane;
            if (k <= len) {
                // source = now - d1 + (k mod d1): always before `now`, so lanes never
                // read a byte this copy writes (and kNear + 273 < kWin: no ring alias)
                const uint32_t r = d1 > len ? k : k % d1;
                const uint32_t v = byte_back(now, d1 - r);
                if (k < len) win[(now + k) & (kWin - 1)] = (uint8_t)v;
                else next = v;
            }
        }
        LANE_FENCE();
        return (uint32_t)__builtin_amdgcn_readlane((int)next, (int)(len % kWave));
    }

    // returns LZMA_OK / LZMA_E_DATA / LZMA_E_OVERFLOW; *now_out = bytes written
    DFI int run(int64_t out_size, uint32_t* now_out) {
        const uint32_t nlit = 0x300u << (lc + lp);
        for (uint32_t i0 = 0; i0 < (uint32_t)PL::COUNT; i0 += kWave)
            if (i0 + lane < (uint32_t)PL::COUNT) probs[i0 + lane] = kBitModelTotal >> 1;
        for (uint32_t i0 = 0; i0 < nlit; i0 += 2 * kWave)   // u32 pairs (nlit is even)
            if (i0 + 2 * lane < nlit) *(uint32_t*)(lit + i0 + 2 * lane) = (kBitModelTotal >> 1) * 0x10001u;
        if (LITP)
            for (uint32_t i0 = 0; i0 < (256u << kDecLitpBits); i0 += 2 * kWave)
                *(uint32_t*)(litp + i0 + 2 * lane) = (kBitModelTotal >> 1) * 0x10001u;
        LANE_FENCE();
        ipos = 0;
        ibase = 0;
        refill(0);
        flushed = 0;
        code = 0;
        range = 0xFFFFFFFFu;
        for (int i = 0; i < 5; i++) code = (code << 8) | rd_byte();   // RangeDecoder.Init
        uint32_t state = 0, rep0 = 0, rep1 = 0, rep2 = 0, rep3 = 0;
        uint32_t mb_next = 0;   // out[now - rep0 - 1] after a copy (the next literal's match byte)
        uint32_t now = 0;
        uint32_t prev = 0;
        int rc = LZMA_OK;
        // out_size >= 0: stop after out_size bytes (capped at 2^32 - 1, beyond any capacity)
        const uint32_t stop = out_size < 0 || out_size > 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)out_size;
        FairPrio prio;   // lzma_common.h: the waves of a CU progress together
        prio.start(g_dec_sched, stop, lane);
        while (out_size < 0 || now < stop) {
            prio.update(now, lane);
            const uint32_t ps = now & ps_mask;
            // literal prefetch, issued before the isMatch decision: the coder's tree
            // (nodes 0-255) and, in matched mode, the 8 nodes along the match byte
            const bool matched = !st_is_char(state);   // only right after a match / rep: copy() left mb
            const uint32_t mb = matched ? mb_next : 0u;
            const uint32_t cidx = ((now & ((1u << lp) - 1)) << lc) + (prev >> (8 - lc));
            uint16_t* sub = lit + (size_t)cidx * 0x300;
            uint16_t* plain = LITP ? litp + cidx * 256u : sub;   // the plain tree (nodes < 0x100)
            T256 tt;
            uint32_t mv[kVS];
            fetch256(plain, tt);
#pragma unroll
            for (int s = 0; s < kVS; s++) {
                const uint32_t i = (uint32_t)(s * kWave) + lane;
                mv[s] = 0;
                if (matched && i < 8) {   // level i: prefix of mb with the leading 1, match bit 7 - i
                    const uint32_t mbit = (mb >> (7 - i)) & 1u;
                    mv[s] = sub[((1 + mbit) << 8) + ((0x100u | mb) >> (8 - i))];
                }
            }
            LANE_FENCE();   // keeps the loads here (not sunk into the literal branch)
            if (bit(probs + PL::IS_MATCH, (state << PBS) + ps) == 0) {
                // LiteralDecoder.Decoder2.DecodeNormal / DecodeWithMatchByte (Decoder.java:67-102)
                uint32_t sym = 1;
                bool same = matched;
                // unrolled: level i's nodes are [2^i, 2^(i+1)), so levels 0-6 read the
                // low lane vector only (a static choice)
                if (!matched) {   // DecodeNormal: no match-byte bookkeeping per bit
#pragma unroll
                    for (uint32_t i = 0; i < 8; i++) {
                        uint32_t np;
                        const uint32_t x = dbit(node256(tt, sym, (int)i), &np);
                        plain[sym] = (uint16_t)np;
                        sym = (sym << 1) | x;
                    }
                } else
#pragma unroll
                for (uint32_t i = 0; i < 8; i++) {
                    uint32_t np, idx, prob;
                    const uint32_t mbit = (mb >> (7 - i)) & 1u;
                    if (same) { idx = ((1 + mbit) << 8) + sym; prob = vget(mv, i); }
                    else {
                        idx = sym;
                        prob = node256(tt, sym, (int)i);
                    }
                    const uint32_t x = dbit(prob, &np);
                    (same ? sub : plain)[idx] = (uint16_t)np;   // every lane, same address and value
                    if (same && x != mbit) same = false;
                    sym = (sym << 1) | x;
                }
                prev = sym & 0xFF;
                if (now >= cap) { rc = LZMA_E_OVERFLOW; break; }
                put(now, prev);
                now++;
                state = st_lit(state);
            } else {
                uint32_t len;
                uint32_t lv[kVS];
                T256 ht;
                if (bit(probs + PL::IS_REP, state) == 1) {
                    fetch_len(probs + PL::RLEN, ps, lv, ht);
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
                    if (len == 0) { len = len_dec(probs + PL::RLEN, ps, lv, ht) + kMatchMinLen; state = st_long(state); }
                } else {
                    fetch_len(probs + PL::LEN, ps, lv, ht);
                    rep3 = rep2; rep2 = rep1; rep1 = rep0;
                    len = kMatchMinLen + len_dec(probs + PL::LEN, ps, lv, ht);
                    state = st_match(state);
                    uint16_t* slot_p = probs + PL::PSLOT + (len_to_pos_state(len) << 6);
                    uint32_t sv[kVS], av[kVS];
                    fetch64(slot_p, 64, sv);
                    fetch64(probs + PL::ALIGN, kAlignTableSize, av);
                    const uint32_t slot = bt_dec(slot_p, sv, kNumPosSlotBits);
                    if (slot >= (uint32_t)kStartPosModelIndex) {
                        uint32_t ndb = (slot >> 1) - 1;
                        rep0 = (2 | (slot & 1)) << ndb;
                        if (slot < (uint32_t)kEndPosModelIndex) {
                            uint16_t* pe = probs + PL::PENC + (int32_t)(rep0 - slot - 1);
                            uint32_t pv[kVS];
                            fetch64(pe, 1u << ndb, pv);
                            rep0 += bt_rev_dec(pe, pv, (int)ndb);
                        } else {
                            rep0 += direct((int)(ndb - kNumAlignBits)) << kNumAlignBits;
                            rep0 += bt_rev_dec(probs + PL::ALIGN, av, kNumAlignBits);
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
                if (rep0 >= now || rep0 >= dict_check) { rc = LZMA_E_DATA; break; }
                const uint32_t d1 = rep0 + 1;
                if ((uint64_t)now + len > cap) {   // copy what fits, then report (no bytes past the capacity)
                    const uint32_t fit = cap - now;
                    copy(now, d1, fit);
                    now = cap;
                    rc = LZMA_E_OVERFLOW;
                    break;
                }
                mb_next = copy(now, d1, len);
                now += len;
                prev = win[(now - 1) & (kWin - 1)];
            }
            maybe_flush(now);
        }
        flush_to(now);
        *now_out = now;
        prio.finish(lane);
        return rc;
    }
};

// LDS of one stream: fixed models, input ring, output window (16-byte aligned regions)
// and (LITP) the plain literal trees
template <int PBS, bool LITP>
constexpr size_t kDecLdsBytes = (((size_t)ProbLayout<PBS>::COUNT * 2 + 15) & ~(size_t)15) + kIbuf + kWin +
                                (LITP ? (size_t)(256u << kDecLitpBits) * 2 : 0);

template <int PBS, bool LITP>
__global__ void __launch_bounds__(kWave) dec_kernel(DecArgs a) {
    // a static LDS array (the layout is fixed per PBS): its address is known when the kernel
    // is compiled, so LDS offsets fold into the ds instructions (a dynamic extern array's
    // base is a link-time constant that costs an s_add per address computation)
    __shared__ __attribute__((aligned(16))) uint8_t smem[kDecLdsBytes<PBS, LITP>];
    Dec<PBS, LITP> d;
    d.lane = threadIdx.x;
    d.lc = a.lc; d.lp = a.lp; d.pb = a.pb; d.ps_mask = (1u << a.pb) - 1; d.dict_check = a.dict_check;
    size_t off = 0;
    auto take = [&](size_t bytes) { uint8_t* p = smem + off; off += (bytes + 15) & ~(size_t)15; return p; };
    d.probs = (uint16_t*)take((size_t)ProbLayout<PBS>::COUNT * 2);
    d.ibuf = take(kIbuf);
    d.win = take(kWin);
    d.litp = LITP ? (uint16_t*)take((size_t)(256u << kDecLitpBits) * 2) : nullptr;
    d.lit = (uint16_t*)(a.scratch + (size_t)blockIdx.x * a.scratch_stride);
    // one workgroup per stream; per-stream values are wave-uniform (readfirstlane keeps them scalar)
    const int s = __builtin_amdgcn_readfirstlane((int)a.order[blockIdx.x]);
    if (s < 0 || s >= a.nstreams) return;   // a corrupt order entry: touch nothing (the host checked the order it wrote)
    const uint64_t i0 = dec_uni64(a.in_offs[s]), o0 = dec_uni64(a.out_offs[s]);
    const uint64_t i1 = dec_uni64(a.in_offs[s + 1]), o1 = dec_uni64(a.out_offs[s + 1]);
    if (i1 < i0 || o1 < o0) {   // offsets the host validated, changed under the kernel: report, do not fault
        if (d.lane == 0) { a.out_lens[s] = 0; a.status[s] = LZMA_E_INTERNAL; }
        return;
    }
    d.in = a.in + i0;
    const uint64_t n_in = i1 - i0, cap = o1 - o0;
    d.n_in = n_in > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)n_in;   // the host rejects inputs >= 4 GiB
    d.out = a.out + o0;
    d.cap = cap > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)cap;
    d.outb = __builtin_amdgcn_make_buffer_rsrc(d.out, 0, d.cap, 0x00020000);
    const int64_t out_size = (int64_t)dec_uni64((uint64_t)a.out_sizes[s]);
    uint32_t now = 0;
    int rc = d.run(out_size, &now);
    if (d.lane == 0) { a.out_lens[s] = now; a.status[s] = rc; }
}

// literal coders of one stream (HBM), 256-byte aligned
size_t dec_scratch_per_block(uint32_t lc, uint32_t lp) { return ((size_t)0x300 << (lc + lp)) * 2 + 256; }

static size_t dec_lds_bytes(uint32_t pb) {
    auto r = [](size_t b) { return (b + 15) & ~(size_t)15; };
    return r((size_t)prob_count(pb) * 2) + r(kIbuf) + r(kWin);
}

int dec_grid(uint32_t, uint32_t, uint32_t, int nstreams) { return nstreams; }   // one workgroup per stream

// The plain literal trees go to LDS only when at most 8 streams share a CU: at 16 per
// CU their 4 KiB each leave too little LDS for the match finder's sorts (24.6 KiB per
// block) that a pipelined caller runs beside the decode (measured: bench step 919 ->
// 994 ms with the sorts 72 -> 162 ms, profiles/r04/bench_dec_litp_16_per_cu.json).
constexpr int kDecLitpMaxStreams = 2048;

template <int PBS>
static void launch_dec(const DecArgs& a, int grid, size_t lds, hipStream_t st) {
    (void)lds;   // static LDS (kDecLdsBytes)
    static const int litp_max = exp_env("LZG_DEC_LITP_MAX") ? atoi(exp_env("LZG_DEC_LITP_MAX")) : kDecLitpMaxStreams;   // experiment build
    if (a.lc + a.lp <= kDecLitpBits && grid <= litp_max)
        hipLaunchKernelGGL((dec_kernel<PBS, true>), dim3(grid), dim3(kWave), 0, st, a);
    else hipLaunchKernelGGL((dec_kernel<PBS, false>), dim3(grid), dim3(kWave), 0, st, a);
}

int launch_decoder(Ctx* ctx, const DecArgs& a, int grid, hipStream_t st) {
    if (a.lit_in_lds || a.scratch == nullptr) return ctx->fail(LZMA_E_INTERNAL, "decoder needs the literal-coder scratch");
    const size_t lds = dec_lds_bytes(a.pb);
    TimedLaunch tl(ctx, "dec_stream", st);
    if (a.pb <= 2) launch_dec<2>(a, grid, lds, st); else launch_dec<4>(a, grid, lds, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "dec launch: %s", hipGetErrorString(e));
    return LZMA_OK;
}

}  // namespace lzg
