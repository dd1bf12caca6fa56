// enc.hip -- phase 2 of the encoder: the price-driven optimal parser and the
// range coder of src/main/java/SevenZip/Compression/LZMA/Encoder.java, one
// wavefront (kWave = 64 lanes) per independent stream.
//
// The parse is strictly serial per stream (adaptive probabilities and the
// price-table refresh schedule depend on every earlier symbol), so the GPU
// gets its throughput from many streams: a persistent grid pulls streams
// from a work queue (longest first). Inside a stream the wave's lanes run the
// data-parallel parts of getOptimum (Encoder.java:364-811):
//   * byte-compare loops (InWindow.GetMatchLen, InWindow.java:120-134): 64
//     bytes per step + ballot,
//   * the per-length price loops for reps and matches (each length updates a
//     distinct _optimum slot, so lanes never collide; the ORDER between reps,
//     pairs and their look-ahead candidates is kept exactly as the reference
//     so strict-< ties resolve identically),
//   * literal prices (8 bit-prices summed across lanes),
//   * the periodic price-table refreshes (FillDistancesPrices,
//     FillAlignPrices, LenPriceTableEncoder.UpdateTable).
// Everything else is wave-uniform scalar code executed by all lanes.
// Probability models, price tables and the first kOptLds _optimum entries
// live in LDS; the match lists come from phase 1 (mf.hip).
#include "lzma_common.h"
#include "runtime.h"

namespace lzg {

static __constant__ Tables c_tab = make_tables();

constexpr int kOptLds = 256;
constexpr int kLitLdsMaxBits = 3;   // literal coders in LDS when lc + lp <= 3
constexpr int kMdCap = kMatchMaxLen + 1;

// Optimal (Optimal.java:3-34); flags bit0 = Prev1IsChar, bit1 = Prev2
struct OptE {
    uint32_t price;
    int32_t pos_prev, back_prev, pos_prev2, back_prev2;
    uint32_t state, flags;
    uint32_t backs[4];
};

#define WSYNC() __syncthreads()

template <typename PairT>
struct Enc {
    using PP = PairPack<PairT>;
    int lane;
    // LDS-resident model and price state
    uint16_t* probs;
    uint16_t* lit;
    uint32_t* pp;
    uint32_t* lenp;         // [2][16 * len_table_size]
    uint32_t* lenc;         // [2][16]
    uint32_t* pos_slot_prices;
    uint32_t* dist_prices;
    uint32_t* align_prices;
    uint32_t* temp_prices;  // [128] FillDistancesPrices scratch
    uint32_t* md_len;
    uint32_t* md_dist;
    OptE* opt_l;
    OptE* opt_g;
    // parameters
    uint32_t fb, lc, lp, pb, ps_mask, eos, dist_table_size, len_table_size;
    // stream
    const uint8_t* in;
    uint32_t n;
    uint8_t* out;
    uint64_t cap, outpos;
    bool overflow;
    const uint32_t* minfo;
    const PairT* pairs;
    const uint32_t* ovf_off;
    const PairT* ovf;
    uint64_t gbase;
    // RangeEncoder (RangeEncoder.java:9-14)
    uint64_t low;
    uint32_t range, cache_size, cache;
    // Encoder fields (Encoder.java:132-181)
    uint32_t mfpos;                 // match-finder position, 0-based (BinTree._pos - 1)
    int32_t additional_offset, opt_end, opt_cur;
    bool longest_found;
    uint32_t longest_len, num_pairs;
    uint32_t state, prev_byte;
    uint32_t rep_dist[4], reps[4], rep_lens[4];
    uint32_t match_price_count, align_price_count;

    __device__ OptE* opt(int32_t i) { return i < kOptLds ? opt_l + i : opt_g + i; }

    // ---- prices (ProbPrices.java:23-36)
    __device__ uint32_t price_bit(uint32_t prob, uint32_t bit) const { return pp[(((prob - bit) ^ (0u - bit)) & 2047u) >> 2]; }
    __device__ uint32_t price0(uint32_t prob) const { return pp[prob >> 2]; }
    __device__ uint32_t price1(uint32_t prob) const { return pp[(kBitModelTotal - prob) >> 2]; }
    __device__ uint32_t bt_price(const uint16_t* p, int nbits, uint32_t sym) const {   // BitTreeEncoder.java:38-48
        uint32_t price = 0, m = 1;
        for (int b = nbits; b != 0;) { b--; uint32_t bit = (sym >> b) & 1; price += price_bit(p[m], bit); m = (m << 1) + bit; }
        return price;
    }
    __device__ uint32_t rev_price(const uint16_t* p, int nbits, uint32_t sym) const {  // BitTreeEncoder.java:50-60
        uint32_t price = 0, m = 1;
        for (int i = nbits; i != 0; i--) { uint32_t bit = sym & 1; sym >>= 1; price += price_bit(p[m], bit); m = (m << 1) | bit; }
        return price;
    }
    __device__ uint16_t* lit_coder(uint32_t pos, uint32_t prev) {   // LiteralEncoder.GetSubCoder (LiteralEncoder.java:93-95)
        uint32_t idx = ((pos & ((1u << lp) - 1)) << lc) + (prev >> (8 - lc));
        return lit + (size_t)idx * 0x300;
    }
    // LiteralEncoder.Encoder2.GetPrice (LiteralEncoder.java:42-64): lanes 0..7 each price one bit.
    __device__ uint32_t lit_price(const uint16_t* p, bool match_mode, uint32_t mb, uint32_t sym) {
        uint32_t price = 0;
        int first = -1;
        if (match_mode) {
            uint32_t diff = (mb ^ sym) & 0xFFu;
            first = diff ? 31 - __clz(diff) : -1;
        }
        for (int j = lane; j < 8; j += kWave) {
            int i = 7 - j;
            uint32_t bit = (sym >> i) & 1;
            uint32_t ctx = (0x100u | sym) >> (i + 1);
            uint32_t idx = ctx;
            if (match_mode && i >= first) idx = ((1 + ((mb >> i) & 1)) << 8) + ctx;
            price += price_bit(p[idx], bit);
        }
        for (int o = 1; o < 8 && o < kWave; o <<= 1) price += __shfl_xor(price, o);
        return __shfl(price, 0);
    }
    __device__ uint32_t len_price(int which, uint32_t sym, uint32_t ps) const {
        return lenp[which * (kNumPosStatesMax * len_table_size) + ps * len_table_size + sym];
    }

    // ---- window access (InWindow.java:115-138), resident stream
    __device__ uint32_t byte_at(int32_t index) const { return in[(int64_t)mfpos + index]; }
    __device__ uint32_t avail() const { return n - mfpos; }
    __device__ uint32_t match_len(int32_t index, uint32_t distance, int32_t limit) const {
        int64_t p0 = (int64_t)mfpos + index;
        if (p0 + limit > (int64_t)n) limit = (int32_t)((int64_t)n - p0);
        if (limit <= 0) return 0;
        const uint8_t* a = in + p0;
        const uint8_t* b = a - ((int64_t)distance + 1);
        for (int32_t i0 = 0; i0 < limit; i0 += kWave) {
            int32_t i = i0 + lane;
            bool ne = i < limit ? (a[i] != b[i]) : true;
            uint64_t m = __ballot(ne);
            if (m) {
                int32_t r = i0 + (__ffsll((long long)m) - 1);
                return (uint32_t)(r < limit ? r : limit);
            }
        }
        return (uint32_t)limit;
    }

    // ---- range encoder (RangeEncoder.java:38-87)
    __device__ void put_byte(uint32_t b) {
        if (outpos < cap) out[outpos] = (uint8_t)b;
        else overflow = true;
        outpos++;
    }
    __device__ void shift_low() {
        uint32_t hi = (uint32_t)(low >> 32);
        if (hi != 0 || low < 0xFF000000ull) {
            uint32_t temp = cache;
            do { put_byte((temp + hi) & 0xFF); temp = 0xFF; } while (--cache_size != 0);
            cache = ((uint32_t)low) >> 24;
        }
        cache_size++;
        low = (low & 0xFFFFFFull) << 8;
    }
    __device__ void rc_bit(uint16_t* p, uint32_t idx, uint32_t bit) {
        uint32_t prob = p[idx];
        uint32_t bound = (range >> 11) * prob;
        if (bit == 0) { range = bound; p[idx] = (uint16_t)(prob + ((kBitModelTotal - prob) >> kNumMoveBits)); }
        else { low += bound; range -= bound; p[idx] = (uint16_t)(prob - (prob >> kNumMoveBits)); }
        if ((range & kTopMask) == 0) { range <<= 8; shift_low(); }
    }
    __device__ void rc_direct(uint32_t v, int nbits) {
        for (int i = nbits - 1; i >= 0; i--) {
            range >>= 1;
            if ((v >> i) & 1) low += range;
            if ((range & kTopMask) == 0) { range <<= 8; shift_low(); }
        }
    }
    __device__ void rc_flush() { for (int i = 0; i < 5; i++) shift_low(); }
    __device__ void bt_enc(uint16_t* p, int nbits, uint32_t sym) {
        uint32_t m = 1;
        for (int b = nbits; b != 0;) { b--; uint32_t bit = (sym >> b) & 1; rc_bit(p, m, bit); m = (m << 1) | bit; }
    }
    __device__ void bt_rev_enc(uint16_t* p, int nbits, uint32_t sym) {
        uint32_t m = 1;
        for (int i = 0; i < nbits; i++) { uint32_t bit = sym & 1; rc_bit(p, m, bit); m = (m << 1) | bit; sym >>= 1; }
    }
    __device__ void lit_encode(uint16_t* p, uint32_t sym) {   // LiteralEncoder.java:17-24
        uint32_t ctx = 1;
        for (int i = 7; i >= 0; i--) { uint32_t bit = (sym >> i) & 1; rc_bit(p, ctx, bit); ctx = (ctx << 1) | bit; }
    }
    __device__ void lit_encode_matched(uint16_t* p, uint32_t mb, uint32_t sym) {   // LiteralEncoder.java:26-40
        uint32_t ctx = 1;
        bool same = true;
        for (int i = 7; i >= 0; i--) {
            uint32_t bit = (sym >> i) & 1, st = ctx;
            if (same) { uint32_t mbit = (mb >> i) & 1; st += (1 + mbit) << 8; same = (mbit == bit); }
            rc_bit(p, st, bit);
            ctx = (ctx << 1) | bit;
        }
    }

    // ---- price tables
    __device__ void update_len_table(int which, uint32_t ps) {   // LenEncoder.SetPrices + LenPriceTableEncoder.UpdateTable
        const uint16_t* L = probs + (which ? P_REP_LEN : P_LEN);
        uint32_t a0 = price0(L[LEN_CHOICE]), a1 = price1(L[LEN_CHOICE]);
        uint32_t b0 = a1 + price0(L[LEN_CHOICE + 1]), b1 = a1 + price1(L[LEN_CHOICE + 1]);
        uint32_t* dst = lenp + which * (kNumPosStatesMax * len_table_size) + ps * len_table_size;
        for (uint32_t i = lane; i < len_table_size; i += kWave) {
            uint32_t pr;
            if (i < kNumLowLenSymbols) pr = a0 + bt_price(L + LEN_LOW + ps * 8, 3, i);
            else if (i < kNumLowLenSymbols + kNumMidLenSymbols) pr = b0 + bt_price(L + LEN_MID + ps * 8, 3, i - kNumLowLenSymbols);
            else pr = b1 + bt_price(L + LEN_HIGH, 8, i - kNumLowLenSymbols - kNumMidLenSymbols);
            dst[i] = pr;
        }
        lenc[which * 16 + ps] = len_table_size;
        WSYNC();
    }
    __device__ void len_encode(int which, uint32_t sym, uint32_t ps) {   // LenEncoder.java:24-39 + LenPriceTableEncoder.java:31-37
        uint16_t* L = probs + (which ? P_REP_LEN : P_LEN);
        if (sym < kNumLowLenSymbols) { rc_bit(L, LEN_CHOICE, 0); bt_enc(L + LEN_LOW + ps * 8, 3, sym); }
        else {
            sym -= kNumLowLenSymbols;
            rc_bit(L, LEN_CHOICE, 1);
            if (sym < kNumMidLenSymbols) { rc_bit(L, LEN_CHOICE + 1, 0); bt_enc(L + LEN_MID + ps * 8, 3, sym); }
            else { rc_bit(L, LEN_CHOICE + 1, 1); bt_enc(L + LEN_HIGH, 8, sym - kNumMidLenSymbols); }
        }
        uint32_t c = lenc[which * 16 + ps] - 1;
        WSYNC();
        lenc[which * 16 + ps] = c;
        if (c == 0) update_len_table(which, ps);
    }
    __device__ void fill_distances_prices() {   // Encoder.java:1087-1118
        for (uint32_t i = kStartPosModelIndex + lane; i < (uint32_t)kNumFullDistances; i += kWave) {
            uint32_t ps = c_tab.fastpos[i], footer = (ps >> 1) - 1, base = (2 | (ps & 1)) << footer;
            temp_prices[i] = rev_price(probs + P_POS_ENC + (int32_t)(base - ps - 1), (int)footer, i - base);
        }
        for (uint32_t l = 0; l < kNumLenToPosStates; l++) {
            uint32_t st = l << kNumPosSlotBits;
            for (uint32_t ps = lane; ps < dist_table_size; ps += kWave) {
                uint32_t pr = bt_price(probs + P_POS_SLOT + st, kNumPosSlotBits, ps);
                if (ps >= (uint32_t)kEndPosModelIndex) pr += (((ps >> 1) - 1) - kNumAlignBits) << 6;
                pos_slot_prices[st + ps] = pr;
            }
        }
        WSYNC();
        for (uint32_t l = 0; l < kNumLenToPosStates; l++) {
            uint32_t st = l << kNumPosSlotBits, st2 = l * kNumFullDistances;
            for (uint32_t i = lane; i < (uint32_t)kNumFullDistances; i += kWave) {
                uint32_t v;
                if (i < (uint32_t)kStartPosModelIndex) v = pos_slot_prices[st + i];
                else v = pos_slot_prices[st + c_tab.fastpos[i]] + temp_prices[i];
                dist_prices[st2 + i] = v;
            }
        }
        match_price_count = 0;
        WSYNC();
    }
    __device__ void fill_align_prices() {   // Encoder.java:1120-1125
        for (uint32_t i = lane; i < (uint32_t)kAlignTableSize; i += kWave) align_prices[i] = rev_price(probs + P_ALIGN, kNumAlignBits, i);
        align_price_count = 0;
        WSYNC();
    }

    // ---- encoder helpers (Encoder.java:275-333)
    __device__ uint32_t read_match_distances() {
        uint64_t g = gbase + mfpos;
        uint32_t info = minfo[g];
        uint32_t cnt = info & 0xFFFFu, ml = info >> 16;
        for (uint32_t k = lane; k < cnt; k += kWave) {
            PairT pr = k < (uint32_t)kInlinePairs ? pairs[g * kInlinePairs + k] : ovf[ovf_off[g] + k - kInlinePairs];
            md_len[k] = PP::len(pr);
            md_dist[k] = PP::dist(pr);
        }
        WSYNC();
        num_pairs = cnt;
        mfpos++;
        additional_offset++;
        return ml;
    }
    __device__ void move_pos(uint32_t num) {
        if (num > 0) { mfpos += num; additional_offset += (int32_t)num; }
    }
    __device__ uint32_t rep_len1_price(uint32_t st, uint32_t ps) const {
        return price0(probs[P_IS_REP_G0 + st]) + price0(probs[P_IS_REP0_LONG + (st << 4) + ps]);
    }
    __device__ uint32_t pure_rep_price(uint32_t ri, uint32_t st, uint32_t ps) const {
        uint32_t price;
        if (ri == 0) {
            price = price0(probs[P_IS_REP_G0 + st]);
            price += price1(probs[P_IS_REP0_LONG + (st << 4) + ps]);
        } else {
            price = price1(probs[P_IS_REP_G0 + st]);
            if (ri == 1) price += price0(probs[P_IS_REP_G1 + st]);
            else { price += price1(probs[P_IS_REP_G1 + st]); price += price_bit(probs[P_IS_REP_G2 + st], ri - 2); }
        }
        return price;
    }
    __device__ uint32_t rep_price(uint32_t ri, uint32_t len, uint32_t st, uint32_t ps) const {
        return len_price(1, len - kMatchMinLen, ps) + pure_rep_price(ri, st, ps);
    }
    __device__ uint32_t pos_len_price(uint32_t pos, uint32_t len, uint32_t ps) const {
        uint32_t price, lps = len_to_pos_state(len);
        if (pos < (uint32_t)kNumFullDistances) price = dist_prices[lps * kNumFullDistances + pos];
        else {
            uint32_t slot2;
            if (pos < (1u << 17)) slot2 = c_tab.fastpos[pos >> 6] + 12;
            else if (pos < (1u << 27)) slot2 = c_tab.fastpos[pos >> 16] + 32;
            else slot2 = c_tab.fastpos[pos >> 26] + 52;
            price = pos_slot_prices[(lps << kNumPosSlotBits) + slot2] + align_prices[pos & kAlignMask];
        }
        return price + len_price(0, len - kMatchMinLen, ps);
    }
    // extend lenEnd: while (lenEnd < target) _optimum[++lenEnd].Price = kIfinityPrice
    __device__ void extend_to(uint32_t& len_end, uint32_t target) {
        if (len_end >= target) return;
        for (uint32_t i = len_end + 1 + lane; i <= target; i += kWave) opt((int32_t)i)->price = kInfinityPrice;
        len_end = target;
        WSYNC();
    }
    // lane-parallel "if (price < opt[slot].Price) update" for slots base+l, l in [lo, hi]
    __device__ void relax_rep(uint32_t base_slot, uint32_t lo, uint32_t hi, uint32_t price0_, uint32_t ps,
                              uint32_t pos_prev, uint32_t ri) {
        for (uint32_t l = lo + lane; l <= hi; l += kWave) {
            uint32_t cl = price0_ + len_price(1, l - 2, ps);
            OptE* o = opt((int32_t)(base_slot + l));
            if (cl < o->price) { o->price = cl; o->pos_prev = (int32_t)pos_prev; o->back_prev = (int32_t)ri; o->flags &= ~1u; }
        }
        WSYNC();
    }

    __device__ uint32_t backward(int32_t* back_res, int32_t cur) {   // Encoder.java:335-362
        opt_end = cur;
        int32_t pos_mem = opt(cur)->pos_prev, back_mem = opt(cur)->back_prev;
        do {
            OptE* oc = opt(cur);
            if (oc->flags & 1u) {
                OptE* om = opt(pos_mem);
                om->back_prev = -1; om->flags &= ~1u;         // MakeAsChar
                om->pos_prev = pos_mem - 1;
                if (oc->flags & 2u) {
                    OptE* om1 = opt(pos_mem - 1);
                    om1->flags &= ~1u;
                    om1->pos_prev = oc->pos_prev2;
                    om1->back_prev = oc->back_prev2;
                }
            }
            int32_t pos_prev = pos_mem, back_cur = back_mem;
            OptE* op = opt(pos_prev);
            back_mem = op->back_prev;
            pos_mem = op->pos_prev;
            op->back_prev = back_cur;
            op->pos_prev = cur;
            cur = pos_prev;
        } while (cur > 0);
        opt_cur = opt(0)->pos_prev;
        *back_res = opt(0)->back_prev;
        WSYNC();
        return (uint32_t)opt_cur;
    }

    // getOptimum (Encoder.java:364-811). Returns length; *back_res = pos.
    __device__ uint32_t get_optimum(uint32_t position, int32_t* back_res) {
        if (opt_end != opt_cur) {
            OptE* oc = opt(opt_cur);
            uint32_t len_res = (uint32_t)(oc->pos_prev - opt_cur);
            *back_res = oc->back_prev;
            opt_cur = oc->pos_prev;
            return len_res;
        }
        opt_cur = opt_end = 0;
        uint32_t len_main;
        if (longest_found) { len_main = longest_len; longest_found = false; }
        else len_main = read_match_distances();
        uint32_t npairs = num_pairs;
        uint32_t num_avail = avail() + 1;
        if (num_avail < 2) { *back_res = -1; return 1; }
        if (num_avail > (uint32_t)kMatchMaxLen) num_avail = kMatchMaxLen;

        uint32_t rep_max = 0;
        for (int i = 0; i < kNumRepDistances; i++) {
            reps[i] = rep_dist[i];
            rep_lens[i] = match_len(-1, reps[i], kMatchMaxLen);
            if (rep_lens[i] > rep_lens[rep_max]) rep_max = (uint32_t)i;
        }
        if (rep_lens[rep_max] >= fb) {
            uint32_t len_res = rep_lens[rep_max];
            *back_res = (int32_t)rep_max;
            move_pos(len_res - 1);
            return len_res;
        }
        if (len_main >= fb) {
            *back_res = (int32_t)(md_dist[npairs - 1] + kNumRepDistances);
            move_pos(len_main - 1);
            return len_main;
        }
        uint32_t cur_byte = byte_at(-1);
        uint32_t match_byte = byte_at((int32_t)(0 - rep_dist[0] - 1 - 1));
        if (len_main < 2 && cur_byte != match_byte && rep_lens[rep_max] < 2) { *back_res = -1; return 1; }

        opt(0)->state = state;
        uint32_t pos_state = position & ps_mask;
        {
            OptE* o1 = opt(1);
            uint32_t p1 = price0(probs[P_IS_MATCH + (state << 4) + pos_state]) +
                          lit_price(lit_coder(position, prev_byte), !st_is_char(state), match_byte, cur_byte);
            uint32_t match_price = price1(probs[P_IS_MATCH + (state << 4) + pos_state]);
            uint32_t rep_match_price = match_price + price1(probs[P_IS_REP + state]);
            int32_t bp = -1;
            if (match_byte == cur_byte) {
                uint32_t srp = rep_match_price + rep_len1_price(state, pos_state);
                if (srp < p1) { p1 = srp; bp = 0; }
            }
            o1->price = p1;
            o1->back_prev = bp;
            o1->flags &= ~1u;
            uint32_t len_end = len_main >= rep_lens[rep_max] ? len_main : rep_lens[rep_max];
            if (len_end < 2) { *back_res = bp; WSYNC(); return 1; }
            o1->pos_prev = 0;
            OptE* o0 = opt(0);
            for (int i = 0; i < 4; i++) o0->backs[i] = reps[i];
            WSYNC();
            for (uint32_t l = 2 + lane; l <= len_end; l += kWave) opt((int32_t)l)->price = kInfinityPrice;
            WSYNC();
            for (uint32_t i = 0; i < (uint32_t)kNumRepDistances; i++) {
                uint32_t rl = rep_lens[i];
                if (rl < 2) continue;
                relax_rep(0, 2, rl, rep_match_price + pure_rep_price(i, state, pos_state), pos_state, 0, i);
            }
            uint32_t normal_match_price = match_price + price0(probs[P_IS_REP + state]);
            uint32_t lstart = rep_lens[0] >= 2 ? rep_lens[0] + 1 : 2;
            if (lstart <= len_main) {
                for (uint32_t l = lstart + lane; l <= len_main; l += kWave) {
                    uint32_t k = 0;
                    while (l > md_len[k]) k++;
                    uint32_t distance = md_dist[k];
                    uint32_t cl = normal_match_price + pos_len_price(distance, l, pos_state);
                    OptE* o = opt((int32_t)l);
                    if (cl < o->price) { o->price = cl; o->pos_prev = 0; o->back_prev = (int32_t)(distance + kNumRepDistances); o->flags &= ~1u; }
                }
                WSYNC();
            }
            return parse_forward(position, back_res, len_end);
        }
    }

    __device__ uint32_t parse_forward(uint32_t position, int32_t* back_res, uint32_t len_end) {
        uint32_t cur = 0;
        for (;;) {
            cur++;
            if (cur == len_end) return backward(back_res, (int32_t)cur);
            uint32_t new_len = read_match_distances();
            uint32_t npairs = num_pairs;
            if (new_len >= fb) {
                longest_len = new_len;
                longest_found = true;
                return backward(back_res, (int32_t)cur);
            }
            position++;
            OptE* oc = opt((int32_t)cur);
            int32_t pos_prev = oc->pos_prev;
            uint32_t st;
            uint32_t ocf = oc->flags;
            if (ocf & 1u) {
                pos_prev--;
                if (ocf & 2u) {
                    st = opt(oc->pos_prev2)->state;
                    if (oc->back_prev2 < kNumRepDistances) st = st_long(st);
                    else st = st_match(st);
                } else st = opt(pos_prev)->state;
                st = st_lit(st);
            } else st = opt(pos_prev)->state;
            if (pos_prev == (int32_t)cur - 1) {
                if (oc->back_prev == 0) st = st_short(st);
                else st = st_lit(st);
            } else {
                int32_t pos;
                if ((ocf & 1u) && (ocf & 2u)) {
                    pos_prev = oc->pos_prev2;
                    pos = oc->back_prev2;
                    st = st_long(st);
                } else {
                    pos = oc->back_prev;
                    if (pos < kNumRepDistances) st = st_long(st);
                    else st = st_match(st);
                }
                OptE* o = opt(pos_prev);
                uint32_t b0 = o->backs[0], b1 = o->backs[1], b2 = o->backs[2], b3 = o->backs[3];
                if (pos < kNumRepDistances) {
                    if (pos == 0) { reps[0] = b0; reps[1] = b1; reps[2] = b2; reps[3] = b3; }
                    else if (pos == 1) { reps[0] = b1; reps[1] = b0; reps[2] = b2; reps[3] = b3; }
                    else if (pos == 2) { reps[0] = b2; reps[1] = b0; reps[2] = b1; reps[3] = b3; }
                    else { reps[0] = b3; reps[1] = b0; reps[2] = b1; reps[3] = b2; }
                } else {
                    reps[0] = (uint32_t)(pos - kNumRepDistances); reps[1] = b0; reps[2] = b1; reps[3] = b2;
                }
            }
            WSYNC();
            oc->state = st;
            for (int i = 0; i < 4; i++) oc->backs[i] = reps[i];
            uint32_t cur_price = oc->price;
            uint32_t cur_byte = byte_at(-1);
            uint32_t match_byte = byte_at((int32_t)(0 - reps[0] - 1 - 1));
            uint32_t pos_state = position & ps_mask;
            uint32_t cur_and1 = cur_price + price0(probs[P_IS_MATCH + (st << 4) + pos_state]) +
                                lit_price(lit_coder(position, byte_at(-2)), !st_is_char(st), match_byte, cur_byte);
            OptE* nx = opt((int32_t)cur + 1);
            bool next_is_char = false;
            if (cur_and1 < nx->price) {
                nx->price = cur_and1; nx->pos_prev = (int32_t)cur; nx->back_prev = -1; nx->flags &= ~1u;
                next_is_char = true;
            }
            uint32_t match_price = cur_price + price1(probs[P_IS_MATCH + (st << 4) + pos_state]);
            uint32_t rep_match_price = match_price + price1(probs[P_IS_REP + st]);
            if (match_byte == cur_byte && !(nx->pos_prev < (int32_t)cur && nx->back_prev == 0)) {
                uint32_t srp = rep_match_price + rep_len1_price(st, pos_state);
                if (srp <= nx->price) {
                    nx->price = srp; nx->pos_prev = (int32_t)cur; nx->back_prev = 0; nx->flags &= ~1u;
                    next_is_char = true;
                }
            }
            WSYNC();
            uint32_t num_avail_full = avail() + 1;
            if ((uint32_t)kNumOpts - 1 - cur < num_avail_full) num_avail_full = kNumOpts - 1 - cur;
            uint32_t num_avail = num_avail_full;
            if (num_avail < 2) continue;
            if (num_avail > fb) num_avail = fb;
            if (!next_is_char && match_byte != cur_byte) {   // literal + rep0
                uint32_t t = num_avail_full - 1 < fb ? num_avail_full - 1 : fb;
                uint32_t lt2 = match_len(0, reps[0], (int32_t)t);
                if (lt2 >= 2) {
                    uint32_t st2 = st_lit(st);
                    uint32_t psn = (position + 1) & ps_mask;
                    uint32_t nrmp = cur_and1 + price1(probs[P_IS_MATCH + (st2 << 4) + psn]) + price1(probs[P_IS_REP + st2]);
                    uint32_t offset = cur + 1 + lt2;
                    extend_to(len_end, offset);
                    uint32_t cl = nrmp + rep_price(0, lt2, st2, psn);
                    OptE* o = opt((int32_t)offset);
                    if (cl < o->price) {
                        o->price = cl; o->pos_prev = (int32_t)cur + 1; o->back_prev = 0;
                        o->flags = (o->flags & ~3u) | 1u;
                    }
                    WSYNC();
                }
            }
            uint32_t start_len = 2;
            for (uint32_t ri = 0; ri < (uint32_t)kNumRepDistances; ri++) {
                uint32_t lt = match_len(-1, reps[ri], (int32_t)num_avail);
                if (lt < 2) continue;
                extend_to(len_end, cur + lt);
                uint32_t base_price = rep_match_price + pure_rep_price(ri, st, pos_state);
                relax_rep(cur, 2, lt, base_price, pos_state, cur, ri);
                if (ri == 0) start_len = lt + 1;
                if (lt < num_avail_full) {
                    uint32_t t = num_avail_full - 1 - lt;
                    if (t > fb) t = fb;
                    uint32_t lt2 = match_len((int32_t)lt, reps[ri], (int32_t)t);
                    if (lt2 >= 2) {
                        uint32_t st2 = st_long(st);
                        uint32_t psn = (position + lt) & ps_mask;
                        uint32_t clcp = rep_match_price + rep_price(ri, lt, st, pos_state) +
                                        price0(probs[P_IS_MATCH + (st2 << 4) + psn]) +
                                        lit_price(lit_coder(position + lt, byte_at((int32_t)lt - 2)), true,
                                                  byte_at((int32_t)lt - 1 - (int32_t)(reps[ri] + 1)), byte_at((int32_t)lt - 1));
                        st2 = st_lit(st2);
                        psn = (position + lt + 1) & ps_mask;
                        uint32_t nmp = clcp + price1(probs[P_IS_MATCH + (st2 << 4) + psn]);
                        uint32_t nrmp = nmp + price1(probs[P_IS_REP + st2]);
                        uint32_t offset = lt + 1 + lt2;
                        extend_to(len_end, cur + offset);
                        uint32_t cl = nrmp + rep_price(0, lt2, st2, psn);
                        OptE* o = opt((int32_t)(cur + offset));
                        if (cl < o->price) {
                            o->price = cl; o->pos_prev = (int32_t)(cur + lt + 1); o->back_prev = 0;
                            o->flags |= 3u; o->pos_prev2 = (int32_t)cur; o->back_prev2 = (int32_t)ri;
                        }
                        WSYNC();
                    }
                }
            }
            if (new_len > num_avail) {
                new_len = num_avail;
                for (npairs = 0; new_len > md_len[npairs]; npairs++) {}
                WSYNC();
                md_len[npairs] = new_len;
                npairs++;
                WSYNC();
            }
            if (new_len >= start_len) {
                uint32_t normal_match_price = match_price + price0(probs[P_IS_REP + st]);
                extend_to(len_end, cur + new_len);
                uint32_t offs = 0;
                while (start_len > md_len[offs]) offs++;
                uint32_t seg_lo = start_len;
                for (;;) {
                    uint32_t seg_hi = md_len[offs];
                    uint32_t cur_back = md_dist[offs];
                    // lengths [seg_lo, seg_hi] all use pair `offs`
                    for (uint32_t l = seg_lo + lane; l <= seg_hi; l += kWave) {
                        uint32_t cl = normal_match_price + pos_len_price(cur_back, l, pos_state);
                        OptE* o = opt((int32_t)(cur + l));
                        if (cl < o->price) {
                            o->price = cl; o->pos_prev = (int32_t)cur; o->back_prev = (int32_t)(cur_back + kNumRepDistances);
                            o->flags &= ~1u;
                        }
                    }
                    WSYNC();
                    uint32_t lt = seg_hi;
                    if (lt < num_avail_full) {
                        uint32_t t = num_avail_full - 1 - lt;
                        if (t > fb) t = fb;
                        uint32_t lt2 = match_len((int32_t)lt, cur_back, (int32_t)t);
                        if (lt2 >= 2) {
                            uint32_t cl = normal_match_price + pos_len_price(cur_back, lt, pos_state);
                            uint32_t st2 = st_match(st);
                            uint32_t psn = (position + lt) & ps_mask;
                            uint32_t clcp = cl + price0(probs[P_IS_MATCH + (st2 << 4) + psn]) +
                                            lit_price(lit_coder(position + lt, byte_at((int32_t)lt - 2)), true,
                                                      byte_at((int32_t)lt - (int32_t)(cur_back + 1) - 1), byte_at((int32_t)lt - 1));
                            st2 = st_lit(st2);
                            psn = (position + lt + 1) & ps_mask;
                            uint32_t nmp = clcp + price1(probs[P_IS_MATCH + (st2 << 4) + psn]);
                            uint32_t nrmp = nmp + price1(probs[P_IS_REP + st2]);
                            uint32_t offset = lt + 1 + lt2;
                            extend_to(len_end, cur + offset);
                            cl = nrmp + rep_price(0, lt2, st2, psn);
                            OptE* o = opt((int32_t)(cur + offset));
                            if (cl < o->price) {
                                o->price = cl; o->pos_prev = (int32_t)(cur + lt + 1); o->back_prev = 0;
                                o->flags |= 3u; o->pos_prev2 = (int32_t)cur;
                                o->back_prev2 = (int32_t)(cur_back + kNumRepDistances);
                            }
                            WSYNC();
                        }
                    }
                    offs++;
                    if (offs == npairs) break;
                    seg_lo = seg_hi + 1;
                }
            }
        }
    }

    // ---- symbol emitters (Encoder.java:938-1024, 818-841)
    __device__ void encode_rep(int32_t pos, uint32_t len, uint32_t ps, uint32_t cs) {
        rc_bit(probs + P_IS_REP, state, 1);
        if (pos == 0) {
            rc_bit(probs + P_IS_REP_G0, state, 0);
            rc_bit(probs + P_IS_REP0_LONG, cs, len == 1 ? 0 : 1);
        } else {
            rc_bit(probs + P_IS_REP_G0, state, 1);
            if (pos == 1) rc_bit(probs + P_IS_REP_G1, state, 0);
            else { rc_bit(probs + P_IS_REP_G1, state, 1); rc_bit(probs + P_IS_REP_G2, state, (uint32_t)pos - 2); }
        }
        if (len == 1) state = st_short(state);
        else { len_encode(1, len - kMatchMinLen, ps); state = st_long(state); }
        uint32_t distance = rep_dist[pos];
        if (pos != 0) {
            for (int k = pos; k >= 1; k--) rep_dist[k] = rep_dist[k - 1];
            rep_dist[0] = distance;
        }
    }
    __device__ void encode_match(int32_t backp, uint32_t len, uint32_t ps) {
        rc_bit(probs + P_IS_REP, state, 0);
        state = st_match(state);
        len_encode(0, len - kMatchMinLen, ps);
        uint32_t pos = (uint32_t)(backp - kNumRepDistances);
        uint32_t slot;
        if (pos < (1u << 11)) slot = c_tab.fastpos[pos];
        else if (pos < (1u << 21)) slot = c_tab.fastpos[pos >> 10] + 20;
        else slot = c_tab.fastpos[pos >> 20] + 40;
        bt_enc(probs + P_POS_SLOT + (len_to_pos_state(len) << 6), kNumPosSlotBits, slot);
        if (slot >= (uint32_t)kStartPosModelIndex) {
            uint32_t footer = (slot >> 1) - 1, base = (2 | (slot & 1)) << footer, red = pos - base;
            if (slot < (uint32_t)kEndPosModelIndex) {
                uint16_t* m = probs + P_POS_ENC + (int32_t)(base - slot - 1);
                uint32_t mm = 1, sym = red;
                for (uint32_t i = 0; i < footer; i++) { uint32_t bit = sym & 1; rc_bit(m, mm, bit); mm = (mm << 1) | bit; sym >>= 1; }
            } else {
                rc_direct(red >> kNumAlignBits, (int)(footer - kNumAlignBits));
                bt_rev_enc(probs + P_ALIGN, kNumAlignBits, red & kAlignMask);
                align_price_count++;
            }
        }
        rep_dist[3] = rep_dist[2]; rep_dist[2] = rep_dist[1]; rep_dist[1] = rep_dist[0]; rep_dist[0] = pos;
        match_price_count++;
    }
    __device__ void flush(uint32_t now_pos) {
        if (eos) {   // WriteEndMarker (Encoder.java:818-835)
            uint32_t ps = now_pos & ps_mask;
            rc_bit(probs + P_IS_MATCH, (state << 4) + ps, 1);
            rc_bit(probs + P_IS_REP, state, 0);
            state = st_match(state);
            len_encode(0, 0, ps);
            bt_enc(probs + P_POS_SLOT + (len_to_pos_state(kMatchMinLen) << 6), kNumPosSlotBits, 63);
            uint32_t red = (1u << 30) - 1;
            rc_direct(red >> kNumAlignBits, 30 - kNumAlignBits);
            bt_rev_enc(probs + P_ALIGN, kNumAlignBits, red & kAlignMask);
        }
        rc_flush();
    }

    __device__ void run() {   // Encoder.Code: SetStreams + CodeOneBlock/encodeOne loop (Encoder.java:843-936, 1046-1077)
        const uint32_t nlit = 0x300u << (lc + lp);
        for (uint32_t i = lane; i < (uint32_t)P_FIXED_COUNT; i += kWave) probs[i] = kBitModelTotal >> 1;
        for (uint32_t i = lane; i < nlit; i += kWave) lit[i] = kBitModelTotal >> 1;
        for (uint32_t i = lane; i < 256; i += kWave) pos_slot_prices[i] = 0;
        WSYNC();
        state = 0; prev_byte = 0;
        for (int i = 0; i < 4; i++) rep_dist[i] = 0;
        low = 0; range = 0xFFFFFFFFu; cache_size = 1; cache = 0; outpos = 0; overflow = false;
        longest_found = false; opt_end = 0; opt_cur = 0; additional_offset = 0;
        longest_len = 0; num_pairs = 0; mfpos = 0;
        match_price_count = 0; align_price_count = 0;
        fill_distances_prices();
        fill_align_prices();
        for (uint32_t ps = 0; ps < (1u << pb); ps++) { update_len_table(0, ps); update_len_table(1, ps); }

        uint32_t now_pos = 0;
        if (avail() == 0) { flush(0); return; }
        read_match_distances();
        rc_bit(probs + P_IS_MATCH, (state << 4) + (now_pos & ps_mask), 0);
        state = st_lit(state);
        {
            uint32_t cb = byte_at(0 - additional_offset);
            lit_encode(lit_coder(now_pos, prev_byte), cb);
            prev_byte = cb;
        }
        additional_offset--;
        now_pos++;
        if (avail() == 0) { flush(now_pos); return; }
        for (;;) {
            int32_t back;
            uint32_t len = get_optimum(now_pos, &back);
            uint32_t ps = now_pos & ps_mask;
            uint32_t cs = (state << 4) + ps;
            if (len == 1 && back == -1) {
                rc_bit(probs + P_IS_MATCH, cs, 0);
                uint32_t cb = byte_at(0 - additional_offset);
                uint16_t* sub = lit_coder(now_pos, prev_byte);
                if (st_is_char(state)) lit_encode(sub, cb);
                else lit_encode_matched(sub, byte_at((int32_t)(0 - rep_dist[0] - 1) - additional_offset), cb);
                prev_byte = cb;
                state = st_lit(state);
            } else {
                rc_bit(probs + P_IS_MATCH, cs, 1);
                if (back < kNumRepDistances) encode_rep(back, len, ps, cs);
                else encode_match(back, len, ps);
                prev_byte = byte_at((int32_t)len - 1 - additional_offset);
            }
            WSYNC();
            additional_offset -= (int32_t)len;
            now_pos += len;
            if (additional_offset == 0) {
                if (match_price_count >= (1u << 7)) fill_distances_prices();
                if (align_price_count >= (uint32_t)kAlignTableSize) fill_align_prices();
                if (avail() == 0) { flush(now_pos); return; }
            }
        }
    }
};

template <typename PairT>
__global__ void __launch_bounds__(kWave) enc_kernel(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    Enc<PairT> e;
    e.lane = threadIdx.x;
    e.fb = a.fb; e.lc = a.lc; e.lp = a.lp; e.pb = a.pb; e.ps_mask = (1u << a.pb) - 1; e.eos = a.eos;
    e.dist_table_size = a.dist_table_size; e.len_table_size = a.len_table_size;
    // carve LDS (offsets multiples of 16)
    size_t off = 0;
    auto take = [&](size_t bytes) { uint8_t* p = smem + off; off += (bytes + 15) & ~(size_t)15; return p; };
    e.pp = (uint32_t*)take(512 * 4);
    e.probs = (uint16_t*)take(P_FIXED_COUNT * 2);
    e.lenp = (uint32_t*)take(2 * kNumPosStatesMax * a.len_table_size * 4);
    e.lenc = (uint32_t*)take(2 * 16 * 4);
    e.pos_slot_prices = (uint32_t*)take(256 * 4);
    e.dist_prices = (uint32_t*)take(512 * 4);
    e.align_prices = (uint32_t*)take(16 * 4);
    e.temp_prices = (uint32_t*)take(kNumFullDistances * 4);
    e.md_len = (uint32_t*)take(kMdCap * 4);
    e.md_dist = (uint32_t*)take(kMdCap * 4);
    e.opt_l = (OptE*)take(kOptLds * sizeof(OptE));
    uint8_t* scratch = a.scratch + blockIdx.x * a.scratch_stride;
    e.opt_g = (OptE*)scratch;
    if (a.lit_in_lds) e.lit = (uint16_t*)take((0x300u << (a.lc + a.lp)) * 2);
    else e.lit = (uint16_t*)(scratch + kNumOpts * sizeof(OptE));
    for (int i = e.lane; i < 512; i += kWave) e.pp[i] = c_tab.prices[i];
    WSYNC();
    e.minfo = a.minfo;
    e.pairs = (const PairT*)a.pairs;
    e.ovf_off = a.ovf_off;
    e.ovf = (const PairT*)a.ovf;
    for (;;) {
        int idx = 0;
        if (e.lane == 0) idx = (int)atomicAdd(a.next, 1u);
        idx = __shfl(idx, 0);
        if (idx >= a.nstreams) break;
        int s = (int)a.order[idx];
        e.gbase = a.offs[s];
        e.n = (uint32_t)(a.offs[s + 1] - e.gbase);
        e.in = a.in + e.gbase;
        e.out = a.out + a.out_offs[s];
        e.cap = a.out_offs[s + 1] - a.out_offs[s];
        e.run();
        if (e.lane == 0) {
            a.out_lens[s] = e.outpos;
            a.status[s] = e.overflow ? LZMA_E_OVERFLOW : LZMA_OK;
        }
        WSYNC();
    }
}

size_t enc_lds_bytes(const EncArgs& a) {
    auto r = [](size_t b) { return (b + 15) & ~(size_t)15; };
    size_t s = r(512 * 4) + r(P_FIXED_COUNT * 2) + r(2 * kNumPosStatesMax * a.len_table_size * 4) + r(2 * 16 * 4) +
               r(256 * 4) + r(512 * 4) + r(16 * 4) + r(kNumFullDistances * 4) + 2 * r(kMdCap * 4) + r(kOptLds * sizeof(OptE));
    if (a.lit_in_lds) s += r((0x300u << (a.lc + a.lp)) * 2);
    return s;
}

size_t enc_scratch_per_block(const Derived& d) {
    return kNumOpts * sizeof(OptE) + ((size_t)0x300 << (d.lc + d.lp)) * 2 + 256;
}

int enc_grid(const Derived& d, int nstreams) {
    EncArgs a{};
    a.lc = d.lc; a.lp = d.lp; a.len_table_size = d.len_table_size;
    a.lit_in_lds = (d.lc + d.lp) <= (uint32_t)kLitLdsMaxBits;
    size_t lds = enc_lds_bytes(a);
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

uint32_t enc_lit_in_lds(const Derived& d) { return (d.lc + d.lp) <= (uint32_t)kLitLdsMaxBits; }

int launch_encoder(Ctx* ctx, const EncArgs& a, bool wide_pairs, int grid, hipStream_t st) {
    size_t lds = enc_lds_bytes(a);
    if (lds > 160 * 1024) return ctx->fail(LZMA_E_PARAM, "encoder LDS %zu too large", lds);
    auto kern = wide_pairs ? (const void*)enc_kernel<uint64_t> : (const void*)enc_kernel<uint32_t>;
    if (lds > 64 * 1024) hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    TimedLaunch tl(ctx, "enc_parse", st);
    if (wide_pairs) hipLaunchKernelGGL(enc_kernel<uint64_t>, dim3(grid), dim3(kWave), lds, st, a);
    else hipLaunchKernelGGL(enc_kernel<uint32_t>, dim3(grid), dim3(kWave), lds, st, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "enc launch: %s", hipGetErrorString(e));
    return LZMA_OK;
}

}  // namespace lzg
