/*
 * lzma_oracle.c -- TEST INFRASTRUCTURE ONLY (see lzma_oracle.h).
 *
 * Plain-C restatement of the reference Java encoder/decoder, function by
 * function. Every routine cites the Java file:line it follows
 * (paths relative to src/main/java/SevenZip/ of rfalke/lzma-java).
 * Java int/long/short semantics are mirrored with explicit uint32_t /
 * uint64_t arithmetic. Window buffering (InWindow.MoveBlock/ReadBlock) is
 * replaced by a fully resident input: the reference keeps at least
 * keepSizeAfter = fb + 274 bytes ahead of the match finder (BinTree.java:100-103,
 * InWindow.java:97-106), which saturates every min() in getOptimum, so the
 * resident model produces the same bits (checked by the -d0 golden, whose
 * 2.9 KB window forces MoveBlock thousands of times in the reference).
 */
#include "lzma_oracle.h"

#include <stdlib.h>
#include <string.h>

#define kNumOpts 4096                 /* Encoder.java:19 */
#define kIfinityPrice 0xFFFFFFFu       /* Encoder.java:22 */
#define kNumRepDistances 4             /* Base.java:4 */
#define kNumStates 12                  /* Base.java:5 */
#define kNumPosSlotBits 6              /* Base.java:42 */
#define kNumLenToPosStates 4           /* Base.java:48 */
#define kMatchMinLen 2                 /* Base.java:50 */
#define kNumAlignBits 4                /* Base.java:60 */
#define kAlignTableSize 16
#define kAlignMask 15
#define kStartPosModelIndex 4          /* Base.java:64 */
#define kEndPosModelIndex 14
#define kNumFullDistances 128          /* Base.java:68 */
#define kNumPosStatesBitsMax 4         /* Base.java:73 */
#define kNumPosStatesMax 16
#define kNumLowLenSymbols 8            /* Base.java:78-84 */
#define kNumMidLenSymbols 8
#define kNumLenSymbols 272
#define kMatchMaxLen 273               /* Base.java:85 */
#define kBitModelTotal 2048            /* RangeBase.java:5 */
#define kNumMoveBits 5                 /* RangeBase.java:7 */
#define kTopMask 0xFF000000u           /* RangeBase.java:6 */
/* BinTree.java:19. A test build lowers it (ORACLE_MAX_VAL_FOR_NORMALIZE, oracle/Makefile
 * `norm`) so that Normalize runs on streams of a few MiB: tests/test_oracle.py pins that it
 * changes no output bit, the premise of the GPU match finder's 1-based
 * absolute positions. */
#ifndef ORACLE_MAX_VAL_FOR_NORMALIZE
#define ORACLE_MAX_VAL_FOR_NORMALIZE ((1u << 30) - 1)
#endif
#define kMaxValForNormalize (ORACLE_MAX_VAL_FOR_NORMALIZE)

/* ------------------------------------------------------------------ tables */
static uint32_t g_crc[256];        /* CRC.java:11-25 */
static uint32_t g_prices[512];     /* ProbPrices.java:8-18 */
static uint8_t g_fast_pos[2048];   /* Encoder.java:30-41 */
static int g_init = 0;

static void init_tables(void) {
    if (g_init) return;
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t r = i;
        for (int j = 0; j < 8; j++) r = (r & 1) ? (r >> 1) ^ 0xEDB88320u : (r >> 1);
        g_crc[i] = r;
    }
    const int kNumBits = 11 - 2;
    for (int i = kNumBits - 1; i >= 0; i--) {
        uint32_t start = 1u << (kNumBits - i - 1), end = 1u << (kNumBits - i);
        for (uint32_t j = start; j < end; j++)
            g_prices[j] = ((uint32_t)i << 6) + (((end - j) << 6) >> (kNumBits - i - 1));
    }
    g_fast_pos[0] = 0;
    g_fast_pos[1] = 1;
    int c = 2;
    for (int slot = 2; slot < 22; slot++) {
        int k = 1 << ((slot >> 1) - 1);
        for (int j = 0; j < k; j++, c++) g_fast_pos[c] = (uint8_t)slot;
    }
    g_init = 1;
}

uint32_t oracle_prob_price(int index) { init_tables(); return g_prices[index & 511]; }

/* ProbPrices.getPrice / GetPrice0 / GetPrice1 (ProbPrices.java:23-36) */
static inline uint32_t price_bit(uint32_t prob, uint32_t bit) {
    return g_prices[(((prob - bit) ^ (0u - bit)) & (kBitModelTotal - 1)) >> 2];
}
static inline uint32_t price0(uint32_t prob) { return g_prices[prob >> 2]; }
static inline uint32_t price1(uint32_t prob) { return g_prices[(kBitModelTotal - prob) >> 2]; }

static void init_probs(uint16_t *p, size_t n) { for (size_t i = 0; i < n; i++) p[i] = kBitModelTotal >> 1; }

/* ------------------------------------------------------------ out buffer */
typedef struct { uint8_t *p; uint64_t n, cap; int oom; } obuf_t;
static void ob_put(obuf_t *o, uint8_t b) {
    if (o->n == o->cap) {
        uint64_t nc = o->cap ? o->cap * 2 : 4096;
        uint8_t *np = (uint8_t *)realloc(o->p, nc);
        if (!np) { o->oom = 1; return; }
        o->p = np; o->cap = nc;
    }
    o->p[o->n++] = b;
}

/* ---------------------------------------------------- RangeEncoder.java */
typedef struct { uint64_t low; uint32_t range, cache_size, cache; uint64_t position; obuf_t *out; } renc_t;

static void re_init(renc_t *r) {            /* RangeEncoder.java:18-24 */
    r->position = 0; r->low = 0; r->range = 0xFFFFFFFFu; r->cache_size = 1; r->cache = 0;
}
static void re_shift_low(renc_t *r) {       /* RangeEncoder.java:73-87 */
    uint32_t low_hi = (uint32_t)(r->low >> 32);
    if (low_hi != 0 || r->low < 0xFF000000ull) {
        r->position += r->cache_size;
        uint32_t temp = r->cache;
        do { ob_put(r->out, (uint8_t)(temp + low_hi)); temp = 0xFF; } while (--r->cache_size != 0);
        r->cache = ((uint32_t)r->low) >> 24;
    }
    r->cache_size++;
    r->low = (r->low & 0xFFFFFFull) << 8;
}
static void re_flush(renc_t *r) { for (int i = 0; i < 5; i++) re_shift_low(r); } /* :31-36 */
static void re_encode(renc_t *r, uint16_t *probs, uint32_t idx, uint32_t bit) { /* :38-54 */
    uint32_t prob = probs[idx];
    uint32_t bound = (r->range >> 11) * prob;
    if (bit == 0) {
        r->range = bound;
        probs[idx] = (uint16_t)(prob + ((kBitModelTotal - prob) >> kNumMoveBits));
    } else {
        r->low += bound;
        r->range -= bound;
        probs[idx] = (uint16_t)(prob - (prob >> kNumMoveBits));
    }
    if ((r->range & kTopMask) == 0) { r->range <<= 8; re_shift_low(r); }
}
static void re_direct_bits(renc_t *r, uint32_t v, int nbits) { /* :56-67 */
    for (int i = nbits - 1; i >= 0; i--) {
        r->range >>= 1;
        if ((v >> i) & 1) r->low += r->range;
        if ((r->range & kTopMask) == 0) { r->range <<= 8; re_shift_low(r); }
    }
}

/* --------------------------------------------------- BitTreeEncoder.java */
static void bt_enc(renc_t *r, uint16_t *probs, int nbits, uint32_t sym) { /* :18-26 */
    uint32_t m = 1;
    for (int b = nbits; b != 0;) { b--; uint32_t bit = (sym >> b) & 1; re_encode(r, probs, m, bit); m = (m << 1) | bit; }
}
static void bt_rev_enc(renc_t *r, uint16_t *probs, int nbits, uint32_t sym) { /* :28-36 */
    uint32_t m = 1;
    for (int i = 0; i < nbits; i++) { uint32_t bit = sym & 1; re_encode(r, probs, m, bit); m = (m << 1) | bit; sym >>= 1; }
}
static uint32_t bt_price(const uint16_t *probs, int nbits, uint32_t sym) { /* :38-48 */
    uint32_t price = 0, m = 1;
    for (int b = nbits; b != 0;) { b--; uint32_t bit = (sym >> b) & 1; price += price_bit(probs[m], bit); m = (m << 1) + bit; }
    return price;
}
static uint32_t bt_rev_price(const uint16_t *probs, int nbits, uint32_t sym) { /* :50-60 */
    uint32_t price = 0, m = 1;
    for (int i = nbits; i != 0; i--) { uint32_t bit = sym & 1; sym >>= 1; price += price_bit(probs[m], bit); m = (m << 1) | bit; }
    return price;
}
/* Encoder.ReverseGetPrice / ReverseEncode (Encoder.java:183-205) */
static uint32_t rev_price_at(const uint16_t *models, int start, int nbits, uint32_t sym) {
    uint32_t price = 0, m = 1;
    for (int i = nbits; i != 0; i--) { uint32_t bit = sym & 1; sym >>= 1; price += price_bit(models[start + m], bit); m = (m << 1) | bit; }
    return price;
}
static void rev_enc_at(renc_t *r, uint16_t *models, int start, int nbits, uint32_t sym) {
    uint32_t m = 1;
    for (int i = 0; i < nbits; i++) { uint32_t bit = sym & 1; re_encode(r, models, start + m, bit); m = (m << 1) | bit; sym >>= 1; }
}

/* ------------------------------------------------------------ Base.java */
static inline uint32_t st_lit(uint32_t s) { return s < 4 ? 0 : (s < 10 ? s - 3 : s - 6); } /* :16-24 */
static inline uint32_t st_match(uint32_t s) { return s < 7 ? 7 : 10; }    /* :26-28 */
static inline uint32_t st_short(uint32_t s) { return s < 7 ? 9 : 11; }    /* :30-32 */
static inline uint32_t st_long(uint32_t s) { return s < 7 ? 8 : 11; }     /* :34-36 */
static inline int st_is_char(uint32_t s) { return s < 7; }                /* :38-40 */
static inline uint32_t len_to_pos_state(uint32_t len) { len -= kMatchMinLen; return len < 4 ? len : 3; } /* :52-58 */

/* Encoder.getPosSlot / GetPosSlot2 (Encoder.java:86-104) */
static inline uint32_t get_pos_slot(uint32_t pos) {
    if (pos < (1u << 11)) return g_fast_pos[pos];
    if (pos < (1u << 21)) return g_fast_pos[pos >> 10] + 20;
    return g_fast_pos[pos >> 20] + 40;
}
static inline uint32_t get_pos_slot2(uint32_t pos) {
    if (pos < (1u << 17)) return g_fast_pos[pos >> 6] + 12;
    if (pos < (1u << 27)) return g_fast_pos[pos >> 16] + 32;
    return g_fast_pos[pos >> 26] + 52;
}

/* --------------------------------------------------------- BinTree.java */
typedef struct {
    const uint8_t *buf;
    int64_t base;                 /* buffer index = base + pos (InWindow._bufferOffset) */
    uint32_t pos, stream_pos;     /* 1-based after reduceOffsets(-1), BinTree.java:79 */
    uint32_t cyc_pos, cyc_size;
    uint32_t match_max_len, cut_value, hash_mask, hash_size_sum, fix_hash_size;
    uint32_t min_match_check, direct_bytes;
    int hash_array;
    uint32_t *son, *hash;
    uint64_t son_cap, hash_cap;   /* allocated entries (kept across streams by a session) */
} bt_t;

/* Create + Init. A session (oracle_enc_new) passes the previous stream's bt_t:
 * like BinTree.Create (BinTree.java:108-133) the arrays are kept when they are
 * large enough, and Init clears the hash heads (BinTree.java:72-80). */
static int bt_create(bt_t *t, const uint8_t *buf, uint64_t n, uint32_t dict, uint32_t fb, int num_hash_bytes) {
    uint32_t *old_son = t->son, *old_hash = t->hash;
    uint64_t old_son_cap = t->son_cap, old_hash_cap = t->hash_cap;
    memset(t, 0, sizeof(*t));
    t->son = old_son; t->hash = old_hash; t->son_cap = old_son_cap; t->hash_cap = old_hash_cap;
    t->buf = buf;
    /* SetType (BinTree.java:59-70) */
    t->hash_array = num_hash_bytes > 2;
    if (t->hash_array) { t->direct_bytes = 0; t->min_match_check = 4; t->fix_hash_size = (1u << 10) + (1u << 16); }
    else { t->direct_bytes = 2; t->min_match_check = 3; t->fix_hash_size = 0; }
    /* Create (BinTree.java:93-134) */
    t->cut_value = 16 + (fb >> 1);
    t->match_max_len = fb;
    /* cyclicBufferSize = dict + 1; for n <= dict the smaller n + 1 gives the
     * same positions (matchMinPos stays 0, cyclicPos = pos - 1). */
    uint64_t cyc = (uint64_t)dict + 1;
    if (n < (uint64_t)dict) cyc = n + 1;
    t->cyc_size = (uint32_t)cyc;
    uint32_t hs = 1u << 16;
    if (t->hash_array) {
        int32_t h = (int32_t)dict - 1;
        h |= (h >> 1); h |= (h >> 2); h |= (h >> 4); h |= (h >> 8);
        h >>= 1;
        h |= 0xFFFF;
        if (h > (1 << 24)) h >>= 1;
        t->hash_mask = (uint32_t)h;
        hs = (uint32_t)h + 1 + t->fix_hash_size;
    }
    t->hash_size_sum = hs;
    if (t->son_cap < (uint64_t)t->cyc_size * 2) {
        free(t->son);
        t->son = (uint32_t *)malloc((size_t)t->cyc_size * 2 * sizeof(uint32_t));
        t->son_cap = t->son ? (uint64_t)t->cyc_size * 2 : 0;
    }
    if (t->hash_cap < hs) {
        free(t->hash);
        t->hash = (uint32_t *)malloc((size_t)hs * sizeof(uint32_t));
        t->hash_cap = t->hash ? hs : 0;
    }
    if (!t->son || !t->hash) return -1;
    memset(t->son, 0, (size_t)t->cyc_size * 2 * sizeof(uint32_t));
    memset(t->hash, 0, (size_t)hs * sizeof(uint32_t));   /* kEmptyHashValue, BinTree.java:76-77 */
    /* Init (BinTree.java:72-80 + InWindow.java:89-95): whole stream resident */
    t->base = -1;
    t->pos = 1;
    t->stream_pos = (uint32_t)n + 1;
    t->cyc_pos = 0;
    return 0;
}
static void bt_free(bt_t *t) { free(t->son); free(t->hash); t->son = t->hash = NULL; t->son_cap = t->hash_cap = 0; }

static uint64_t g_normalize_calls;           /* how often Normalize ran (tests) */
uint64_t oracle_normalize_count(void) { return g_normalize_calls; }
static void bt_normalize(bt_t *t) {          /* BinTree.java:358-375 */
    g_normalize_calls++;
    uint32_t sub = t->pos - t->cyc_size;
    for (uint64_t i = 0; i < (uint64_t)t->cyc_size * 2; i++) { uint32_t v = t->son[i]; t->son[i] = v <= sub ? 0 : v - sub; }
    for (uint32_t i = 0; i < t->hash_size_sum; i++) { uint32_t v = t->hash[i]; t->hash[i] = v <= sub ? 0 : v - sub; }
    t->base += sub; t->pos -= sub; t->stream_pos -= sub;   /* InWindow.reduceOffsets :108-113 */
}
static void bt_inc(bt_t *t) {                /* BinTree.java:82-91 */
    if (++t->cyc_pos >= t->cyc_size) t->cyc_pos = 0;
    t->pos++;
    if (t->pos == kMaxValForNormalize) bt_normalize(t);
}
static inline uint32_t bt_avail(const bt_t *t) { return t->stream_pos - t->pos; } /* InWindow.java:136-138 */
static inline uint8_t bt_byte(const bt_t *t, int32_t index) { return t->buf[t->base + t->pos + index]; } /* :115-117 */

static uint32_t bt_match_len(const bt_t *t, int32_t index, uint32_t distance, int32_t limit) { /* InWindow.java:120-134 */
    int64_t p0 = (int64_t)t->pos + index;
    if (p0 + limit > (int64_t)t->stream_pos) limit = (int32_t)((int64_t)t->stream_pos - p0);
    int64_t d = (int64_t)distance + 1;
    const uint8_t *p = t->buf + (t->base + p0);
    int32_t i;
    for (i = 0; i < limit && p[i] == p[i - d]; i++) {}
    return (uint32_t)i;
}

/* fillMatches0 (BinTree.java:152-273) */
static uint32_t bt_get_matches(bt_t *t, uint32_t *lens, uint32_t *dists) {
    uint32_t len_limit;
    if (t->pos + t->match_max_len <= t->stream_pos) len_limit = t->match_max_len;
    else {
        len_limit = t->stream_pos - t->pos;
        if (len_limit < t->min_match_check) { bt_inc(t); return 0; }
    }
    const uint32_t pos = t->pos;
    uint32_t match_min = pos > t->cyc_size ? pos - t->cyc_size : 0;
    const uint8_t *cur = t->buf + (t->base + pos);
    const uint8_t *bb = t->buf + t->base;      /* bb[p] = byte at 1-based position p */
    uint32_t hv, h2 = 0, h3 = 0;
    if (t->hash_array) {
        uint32_t temp = g_crc[cur[0]] ^ cur[1];
        h2 = temp & 1023u;
        temp ^= (uint32_t)cur[2] << 8;
        h3 = temp & 0xFFFFu;
        hv = (temp ^ (g_crc[cur[3]] << 5)) & t->hash_mask;
    } else {
        hv = cur[0] ^ ((uint32_t)cur[1] << 8);
    }
    uint32_t cur_match = t->hash[t->fix_hash_size + hv];
    uint32_t max_len = 1;
    uint32_t off = 0;
    if (t->hash_array) {
        uint32_t cm2 = t->hash[h2];
        uint32_t cm3 = t->hash[1024 + h3];
        t->hash[h2] = pos;
        t->hash[1024 + h3] = pos;
        if (cm2 > match_min && bb[cm2] == cur[0]) { max_len = 2; lens[off] = 2; dists[off++] = pos - cm2 - 1; }
        if (cm3 > match_min && bb[cm3] == cur[0]) {
            if (cm3 == cm2) off--;
            max_len = 3; lens[off] = 3; dists[off++] = pos - cm3 - 1;
            cm2 = cm3;
        }
        if (off != 0 && cm2 == cur_match) { off--; max_len = 1; }
    }
    t->hash[t->fix_hash_size + hv] = pos;
    uint32_t ptr0 = (t->cyc_pos << 1) + 1, ptr1 = t->cyc_pos << 1;
    uint32_t len0 = t->direct_bytes, len1 = t->direct_bytes;
    if (t->direct_bytes != 0 && cur_match > match_min) {
        if (bb[cur_match + t->direct_bytes] != cur[t->direct_bytes]) {
            max_len = t->direct_bytes; lens[off] = t->direct_bytes; dists[off++] = pos - cur_match - 1;
        }
    }
    uint32_t count = t->cut_value;
    for (;;) {
        if (cur_match <= match_min || count-- == 0) { t->son[ptr0] = 0; t->son[ptr1] = 0; break; }
        uint32_t delta = pos - cur_match;
        uint32_t cp = ((delta <= t->cyc_pos) ? (t->cyc_pos - delta) : (t->cyc_pos - delta + t->cyc_size)) << 1;
        const uint8_t *pby = bb + cur_match;
        uint32_t len = len0 < len1 ? len0 : len1;
        if (pby[len] == cur[len]) {
            while (++len != len_limit) if (pby[len] != cur[len]) break;
            if (max_len < len) {
                max_len = len; lens[off] = len; dists[off++] = delta - 1;
                if (len == len_limit) { t->son[ptr1] = t->son[cp]; t->son[ptr0] = t->son[cp + 1]; break; }
            }
        }
        if (pby[len] < cur[len]) { t->son[ptr1] = cur_match; ptr1 = cp + 1; cur_match = t->son[ptr1]; len1 = len; }
        else { t->son[ptr0] = cur_match; ptr0 = cp; cur_match = t->son[ptr0]; len0 = len; }
    }
    bt_inc(t);
    return off;
}

/* Skip (BinTree.java:275-356) */
static void bt_skip(bt_t *t, uint32_t num) {
    do {
        uint32_t len_limit;
        if (t->pos + t->match_max_len <= t->stream_pos) len_limit = t->match_max_len;
        else {
            len_limit = t->stream_pos - t->pos;
            if (len_limit < t->min_match_check) { bt_inc(t); continue; }
        }
        const uint32_t pos = t->pos;
        uint32_t match_min = pos > t->cyc_size ? pos - t->cyc_size : 0;
        const uint8_t *cur = t->buf + (t->base + pos);
        const uint8_t *bb = t->buf + t->base;
        uint32_t hv;
        if (t->hash_array) {
            uint32_t temp = g_crc[cur[0]] ^ cur[1];
            t->hash[temp & 1023u] = pos;
            temp ^= (uint32_t)cur[2] << 8;
            t->hash[1024 + (temp & 0xFFFFu)] = pos;
            hv = (temp ^ (g_crc[cur[3]] << 5)) & t->hash_mask;
        } else {
            hv = cur[0] ^ ((uint32_t)cur[1] << 8);
        }
        uint32_t cur_match = t->hash[t->fix_hash_size + hv];
        t->hash[t->fix_hash_size + hv] = pos;
        uint32_t ptr0 = (t->cyc_pos << 1) + 1, ptr1 = t->cyc_pos << 1;
        uint32_t len0 = t->direct_bytes, len1 = t->direct_bytes;
        uint32_t count = t->cut_value;
        for (;;) {
            if (cur_match <= match_min || count-- == 0) { t->son[ptr0] = 0; t->son[ptr1] = 0; break; }
            uint32_t delta = pos - cur_match;
            uint32_t cp = ((delta <= t->cyc_pos) ? (t->cyc_pos - delta) : (t->cyc_pos - delta + t->cyc_size)) << 1;
            const uint8_t *pby = bb + cur_match;
            uint32_t len = len0 < len1 ? len0 : len1;
            if (pby[len] == cur[len]) {
                while (++len != len_limit) if (pby[len] != cur[len]) break;
                if (len == len_limit) { t->son[ptr1] = t->son[cp]; t->son[ptr0] = t->son[cp + 1]; break; }
            }
            if (pby[len] < cur[len]) { t->son[ptr1] = cur_match; ptr1 = cp + 1; cur_match = t->son[ptr1]; len1 = len; }
            else { t->son[ptr0] = cur_match; ptr0 = cp; cur_match = t->son[ptr0]; len0 = len; }
        }
        bt_inc(t);
    } while (--num != 0);
}

/* ------------------------------------------------------- LenEncoder.java */
typedef struct {
    uint16_t choice[2];
    uint16_t low[kNumPosStatesMax][1 << 3];
    uint16_t mid[kNumPosStatesMax][1 << 3];
    uint16_t high[1 << 8];
    uint32_t prices[kNumPosStatesMax * kNumLenSymbols];  /* LenPriceTableEncoder.java:4 */
    uint32_t counters[kNumPosStatesMax];
    uint32_t table_size;
} lenenc_t;

static void len_init(lenenc_t *l, uint32_t num_pos_states) { /* LenEncoder.java:14-22 */
    init_probs(l->choice, 2);
    for (uint32_t ps = 0; ps < num_pos_states; ps++) { init_probs(l->low[ps], 8); init_probs(l->mid[ps], 8); }
    init_probs(l->high, 256);
}
static void len_encode_raw(lenenc_t *l, renc_t *r, uint32_t sym, uint32_t ps) { /* LenEncoder.java:24-39 */
    if (sym < kNumLowLenSymbols) { re_encode(r, l->choice, 0, 0); bt_enc(r, l->low[ps], 3, sym); }
    else {
        sym -= kNumLowLenSymbols;
        re_encode(r, l->choice, 0, 1);
        if (sym < kNumMidLenSymbols) { re_encode(r, l->choice, 1, 0); bt_enc(r, l->mid[ps], 3, sym); }
        else { re_encode(r, l->choice, 1, 1); bt_enc(r, l->high, 8, sym - kNumMidLenSymbols); }
    }
}
static void len_set_prices(lenenc_t *l, uint32_t ps, uint32_t num_symbols, uint32_t *prices) { /* LenEncoder.java:41-62 */
    uint32_t a0 = price0(l->choice[0]), a1 = price1(l->choice[0]);
    uint32_t b0 = a1 + price0(l->choice[1]), b1 = a1 + price1(l->choice[1]);
    uint32_t i;
    for (i = 0; i < kNumLowLenSymbols; i++) { if (i >= num_symbols) return; prices[i] = a0 + bt_price(l->low[ps], 3, i); }
    for (; i < kNumLowLenSymbols + kNumMidLenSymbols; i++) { if (i >= num_symbols) return; prices[i] = b0 + bt_price(l->mid[ps], 3, i - kNumLowLenSymbols); }
    for (; i < num_symbols; i++) prices[i] = b1 + bt_price(l->high, 8, i - kNumLowLenSymbols - kNumMidLenSymbols);
}
static void len_update_table(lenenc_t *l, uint32_t ps) { /* LenPriceTableEncoder.java:20-23 */
    len_set_prices(l, ps, l->table_size, l->prices + ps * kNumLenSymbols);
    l->counters[ps] = l->table_size;
}
static void len_encode(lenenc_t *l, renc_t *r, uint32_t sym, uint32_t ps) { /* LenPriceTableEncoder.java:31-37 */
    len_encode_raw(l, r, sym, ps);
    if (--l->counters[ps] == 0) len_update_table(l, ps);
}
static inline uint32_t len_price(const lenenc_t *l, uint32_t sym, uint32_t ps) { return l->prices[ps * kNumLenSymbols + sym]; }

/* ----------------------------------------------------------- Optimal.java */
typedef struct {
    uint32_t state;
    int prev1_is_char, prev2;
    int32_t pos_prev2, back_prev2;
    uint32_t price;
    int32_t pos_prev, back_prev;
    int32_t backs[4];
} optimal_t;

/* ----------------------------------------------------------- Encoder.java */
typedef struct {
    oracle_params prm;
    int mode;
    bt_t bt;
    /* two-phase mode: precomputed lists (mode 1) */
    const uint32_t *pre_counts, *pre_main, *pre_lens, *pre_dists;
    const uint64_t *pre_offs;
    renc_t rc;
    obuf_t out;
    optimal_t opt[kNumOpts];
    uint16_t is_match[kNumStates << kNumPosStatesBitsMax];
    uint16_t is_rep[kNumStates], is_rep_g0[kNumStates], is_rep_g1[kNumStates], is_rep_g2[kNumStates];
    uint16_t is_rep0_long[kNumStates << kNumPosStatesBitsMax];
    uint16_t pos_slot[kNumLenToPosStates][1 << kNumPosSlotBits];
    uint16_t pos_encoders[kNumFullDistances - kEndPosModelIndex];
    uint16_t pos_align[1 << kNumAlignBits];
    lenenc_t len_enc, rep_len_enc;
    uint16_t *lit;     /* (1 << (lc + lp)) x 0x300, LiteralEncoder.java:67-91 */
    uint32_t md_len[kMatchMaxLen + 1], md_dist[kMatchMaxLen + 1];
    uint32_t match_price_count, align_price_count;
    uint32_t num_fast_bytes, longest_match_len, num_distance_pairs;
    int longest_match_found;
    int32_t additional_offset;
    int32_t optimum_end, optimum_cur;
    uint32_t pos_slot_prices[1 << (kNumPosSlotBits + 2)];
    uint32_t distances_prices[kNumFullDistances << 2];
    uint32_t align_prices[kAlignTableSize];
    uint32_t temp_prices[kNumFullDistances];
    uint32_t dist_table_size;
    uint32_t pos_state_bits, pos_state_mask, lp, lc;
    uint32_t state;
    uint8_t previous_byte;
    uint32_t rep_distances[4], reps[4], rep_lens[4];
} enc_t;

/* LiteralEncoder.GetSubCoder (LiteralEncoder.java:93-95) */
static inline uint16_t *lit_coder(enc_t *e, uint32_t pos, uint8_t prev) {
    uint32_t idx = ((pos & ((1u << e->lp) - 1)) << e->lc) + ((uint32_t)prev >> (8 - e->lc));
    return e->lit + (size_t)idx * 0x300;
}
static void lit_encode(renc_t *r, uint16_t *p, uint8_t sym) { /* LiteralEncoder.java:17-24 */
    uint32_t ctx = 1;
    for (int i = 7; i >= 0; i--) { uint32_t bit = (sym >> i) & 1; re_encode(r, p, ctx, bit); ctx = (ctx << 1) | bit; }
}
static void lit_encode_matched(renc_t *r, uint16_t *p, uint8_t mb, uint8_t sym) { /* :26-40 */
    uint32_t ctx = 1; int same = 1;
    for (int i = 7; i >= 0; i--) {
        uint32_t bit = (sym >> i) & 1, st = ctx;
        if (same) { uint32_t mbit = (mb >> i) & 1; st += (1 + mbit) << 8; same = (mbit == bit); }
        re_encode(r, p, st, bit);
        ctx = (ctx << 1) | bit;
    }
}
static uint32_t lit_price(const uint16_t *p, int match_mode, uint8_t mb, uint8_t sym) { /* :42-64 */
    uint32_t price = 0, ctx = 1;
    int i = 7;
    if (match_mode) {
        for (; i >= 0; i--) {
            uint32_t mbit = (mb >> i) & 1, bit = (sym >> i) & 1;
            price += price_bit(p[((1 + mbit) << 8) + ctx], bit);
            ctx = (ctx << 1) | bit;
            if (mbit != bit) { i--; break; }
        }
    }
    for (; i >= 0; i--) { uint32_t bit = (sym >> i) & 1; price += price_bit(p[ctx], bit); ctx = (ctx << 1) | bit; }
    return price;
}

static void fill_distances_prices(enc_t *e) { /* Encoder.java:1087-1118 */
    for (uint32_t i = kStartPosModelIndex; i < kNumFullDistances; i++) {
        uint32_t ps = get_pos_slot(i), fb = (ps >> 1) - 1, base = (2 | (ps & 1)) << fb;
        e->temp_prices[i] = rev_price_at(e->pos_encoders, (int)(base - ps - 1), (int)fb, i - base);
    }
    for (uint32_t l = 0; l < kNumLenToPosStates; l++) {
        uint32_t st = l << kNumPosSlotBits, ps;
        for (ps = 0; ps < e->dist_table_size; ps++) e->pos_slot_prices[st + ps] = bt_price(e->pos_slot[l], kNumPosSlotBits, ps);
        for (ps = kEndPosModelIndex; ps < e->dist_table_size; ps++) e->pos_slot_prices[st + ps] += (((ps >> 1) - 1) - kNumAlignBits) << 6;
        uint32_t st2 = l * kNumFullDistances, i;
        for (i = 0; i < kStartPosModelIndex; i++) e->distances_prices[st2 + i] = e->pos_slot_prices[st + i];
        for (; i < kNumFullDistances; i++) e->distances_prices[st2 + i] = e->pos_slot_prices[st + get_pos_slot(i)] + e->temp_prices[i];
    }
    e->match_price_count = 0;
}
static void fill_align_prices(enc_t *e) { /* Encoder.java:1120-1125 */
    for (uint32_t i = 0; i < kAlignTableSize; i++) e->align_prices[i] = bt_rev_price(e->pos_align, kNumAlignBits, i);
    e->align_price_count = 0;
}

/* match finder access: reference order (mode 0) or precomputed (mode 1) */
static uint32_t mf_get_matches(enc_t *e) {
    if (e->mode == 0) return bt_get_matches(&e->bt, e->md_len, e->md_dist);
    uint64_t idx = e->bt.pos - 1;  /* 0-based position (no Normalize below 2^30) */
    uint32_t c = e->pre_counts[idx];
    for (uint32_t k = 0; k < c; k++) { e->md_len[k] = e->pre_lens[e->pre_offs[idx] + k]; e->md_dist[k] = e->pre_dists[e->pre_offs[idx] + k]; }
    bt_inc(&e->bt);
    return c;
}
static void mf_skip(enc_t *e, uint32_t num) {
    if (e->mode == 0) { bt_skip(&e->bt, num); return; }
    do { bt_inc(&e->bt); } while (--num != 0);
}

static uint32_t read_match_distances(enc_t *e) { /* Encoder.java:275-287 */
    e->num_distance_pairs = mf_get_matches(e);
    uint32_t length = 0;
    if (e->num_distance_pairs > 0) {
        length = e->md_len[e->num_distance_pairs - 1];
        if (length == e->num_fast_bytes)
            length += bt_match_len(&e->bt, (int32_t)length - 1, e->md_dist[e->num_distance_pairs - 1], (int32_t)(kMatchMaxLen - length));
    }
    e->additional_offset++;
    return length;
}
static void move_pos(enc_t *e, uint32_t num) { /* Encoder.java:289-294 */
    if (num > 0) { mf_skip(e, num); e->additional_offset += num; }
}
static inline uint32_t get_rep_len1_price(enc_t *e, uint32_t state, uint32_t ps) { /* :296-299 */
    return price0(e->is_rep_g0[state]) + price0(e->is_rep0_long[(state << kNumPosStatesBitsMax) + ps]);
}
static inline uint32_t get_pure_rep_price(enc_t *e, uint32_t ri, uint32_t state, uint32_t ps) { /* :301-316 */
    uint32_t price;
    if (ri == 0) {
        price = price0(e->is_rep_g0[state]);
        price += price1(e->is_rep0_long[(state << kNumPosStatesBitsMax) + ps]);
    } else {
        price = price1(e->is_rep_g0[state]);
        if (ri == 1) price += price0(e->is_rep_g1[state]);
        else { price += price1(e->is_rep_g1[state]); price += price_bit(e->is_rep_g2[state], ri - 2); }
    }
    return price;
}
static inline uint32_t get_rep_price(enc_t *e, uint32_t ri, uint32_t len, uint32_t state, uint32_t ps) { /* :318-321 */
    return len_price(&e->rep_len_enc, len - kMatchMinLen, ps) + get_pure_rep_price(e, ri, state, ps);
}
static inline uint32_t get_pos_len_price(enc_t *e, uint32_t pos, uint32_t len, uint32_t ps) { /* :323-333 */
    uint32_t price, lps = len_to_pos_state(len);
    if (pos < kNumFullDistances) price = e->distances_prices[lps * kNumFullDistances + pos];
    else price = e->pos_slot_prices[(lps << kNumPosSlotBits) + get_pos_slot2(pos)] + e->align_prices[pos & kAlignMask];
    return price + len_price(&e->len_enc, len - kMatchMinLen, ps);
}
static inline void make_as_char(optimal_t *o) { o->back_prev = -1; o->prev1_is_char = 0; }
static inline void make_as_short_rep(optimal_t *o) { o->back_prev = 0; o->prev1_is_char = 0; }

static uint32_t backward(enc_t *e, int32_t *back_res, int32_t cur) { /* Encoder.java:335-362 */
    e->optimum_end = cur;
    int32_t pos_mem = e->opt[cur].pos_prev, back_mem = e->opt[cur].back_prev;
    do {
        if (e->opt[cur].prev1_is_char) {
            make_as_char(&e->opt[pos_mem]);
            e->opt[pos_mem].pos_prev = pos_mem - 1;
            if (e->opt[cur].prev2) {
                e->opt[pos_mem - 1].prev1_is_char = 0;
                e->opt[pos_mem - 1].pos_prev = e->opt[cur].pos_prev2;
                e->opt[pos_mem - 1].back_prev = e->opt[cur].back_prev2;
            }
        }
        int32_t pos_prev = pos_mem, back_cur = back_mem;
        back_mem = e->opt[pos_prev].back_prev;
        pos_mem = e->opt[pos_prev].pos_prev;
        e->opt[pos_prev].back_prev = back_cur;
        e->opt[pos_prev].pos_prev = cur;
        cur = pos_prev;
    } while (cur > 0);
    e->optimum_cur = e->opt[0].pos_prev;
    *back_res = e->opt[0].back_prev;
    return (uint32_t)e->optimum_cur;
}

/* getOptimum (Encoder.java:364-811). Returns length; *back_res = pos. */
static uint32_t get_optimum(enc_t *e, uint32_t position, int32_t *back_res) {
    optimal_t *opt = e->opt;
    if (e->optimum_end != e->optimum_cur) {
        uint32_t len_res = (uint32_t)(opt[e->optimum_cur].pos_prev - e->optimum_cur);
        *back_res = opt[e->optimum_cur].back_prev;
        e->optimum_cur = opt[e->optimum_cur].pos_prev;
        return len_res;
    }
    e->optimum_cur = e->optimum_end = 0;
    uint32_t len_main;
    if (e->longest_match_found) { len_main = e->longest_match_len; e->longest_match_found = 0; }
    else len_main = read_match_distances(e);
    uint32_t num_distance_pairs = e->num_distance_pairs;
    uint32_t num_avail = bt_avail(&e->bt) + 1;
    if (num_avail < 2) { *back_res = -1; return 1; }
    if (num_avail > kMatchMaxLen) num_avail = kMatchMaxLen;

    uint32_t rep_max = 0, i;
    for (i = 0; i < kNumRepDistances; i++) {
        e->reps[i] = e->rep_distances[i];
        e->rep_lens[i] = bt_match_len(&e->bt, -1, e->reps[i], kMatchMaxLen);
        if (e->rep_lens[i] > e->rep_lens[rep_max]) rep_max = i;
    }
    if (e->rep_lens[rep_max] >= e->num_fast_bytes) {
        uint32_t len_res = e->rep_lens[rep_max];
        *back_res = (int32_t)rep_max;
        move_pos(e, len_res - 1);
        return len_res;
    }
    if (len_main >= e->num_fast_bytes) {
        *back_res = (int32_t)(e->md_dist[num_distance_pairs - 1] + kNumRepDistances);
        move_pos(e, len_main - 1);
        return len_main;
    }
    uint8_t cur_byte = bt_byte(&e->bt, -1);
    uint8_t match_byte = bt_byte(&e->bt, (int32_t)(0 - e->rep_distances[0] - 1 - 1));
    if (len_main < 2 && cur_byte != match_byte && e->rep_lens[rep_max] < 2) { *back_res = -1; return 1; }

    opt[0].state = e->state;
    uint32_t pos_state = position & e->pos_state_mask;
    opt[1].price = price0(e->is_match[(e->state << kNumPosStatesBitsMax) + pos_state]) +
                   lit_price(lit_coder(e, position, e->previous_byte), !st_is_char(e->state), match_byte, cur_byte);
    make_as_char(&opt[1]);
    uint32_t match_price = price1(e->is_match[(e->state << kNumPosStatesBitsMax) + pos_state]);
    uint32_t rep_match_price = match_price + price1(e->is_rep[e->state]);
    if (match_byte == cur_byte) {
        uint32_t short_rep_price = rep_match_price + get_rep_len1_price(e, e->state, pos_state);
        if (short_rep_price < opt[1].price) { opt[1].price = short_rep_price; make_as_short_rep(&opt[1]); }
    }
    uint32_t len_end = len_main >= e->rep_lens[rep_max] ? len_main : e->rep_lens[rep_max];
    if (len_end < 2) { *back_res = opt[1].back_prev; return 1; }
    opt[1].pos_prev = 0;
    for (i = 0; i < 4; i++) opt[0].backs[i] = (int32_t)e->reps[i];
    uint32_t len = len_end;
    do { opt[len--].price = kIfinityPrice; } while (len >= 2);

    for (i = 0; i < kNumRepDistances; i++) {
        uint32_t rep_len = e->rep_lens[i];
        if (rep_len < 2) continue;
        uint32_t price = rep_match_price + get_pure_rep_price(e, i, e->state, pos_state);
        do {
            uint32_t cl = price + len_price(&e->rep_len_enc, rep_len - 2, pos_state);
            optimal_t *o = &opt[rep_len];
            if (cl < o->price) { o->price = cl; o->pos_prev = 0; o->back_prev = (int32_t)i; o->prev1_is_char = 0; }
        } while (--rep_len >= 2);
    }
    uint32_t normal_match_price = match_price + price0(e->is_rep[e->state]);
    len = e->rep_lens[0] >= 2 ? e->rep_lens[0] + 1 : 2;
    if (len <= len_main) {
        uint32_t offs = 0;
        while (len > e->md_len[offs]) offs++;
        for (;; len++) {
            uint32_t distance = e->md_dist[offs];
            uint32_t cl = normal_match_price + get_pos_len_price(e, distance, len, pos_state);
            optimal_t *o = &opt[len];
            if (cl < o->price) { o->price = cl; o->pos_prev = 0; o->back_prev = (int32_t)(distance + kNumRepDistances); o->prev1_is_char = 0; }
            if (len == e->md_len[offs]) { offs++; if (offs == num_distance_pairs) break; }
        }
    }

    uint32_t cur = 0;
    for (;;) {
        cur++;
        if (cur == len_end) return backward(e, back_res, (int32_t)cur);
        uint32_t new_len = read_match_distances(e);
        num_distance_pairs = e->num_distance_pairs;
        if (new_len >= e->num_fast_bytes) {
            e->longest_match_len = new_len;
            e->longest_match_found = 1;
            return backward(e, back_res, (int32_t)cur);
        }
        position++;
        int32_t pos_prev = opt[cur].pos_prev;
        uint32_t state;
        if (opt[cur].prev1_is_char) {
            pos_prev--;
            if (opt[cur].prev2) {
                state = opt[opt[cur].pos_prev2].state;
                if (opt[cur].back_prev2 < kNumRepDistances) state = st_long(state);
                else state = st_match(state);
            } else state = opt[pos_prev].state;
            state = st_lit(state);
        } else state = opt[pos_prev].state;
        if (pos_prev == (int32_t)cur - 1) {
            if (opt[cur].back_prev == 0) state = st_short(state);   /* isShortRep */
            else state = st_lit(state);
        } else {
            int32_t pos;
            if (opt[cur].prev1_is_char && opt[cur].prev2) {
                pos_prev = opt[cur].pos_prev2;
                pos = opt[cur].back_prev2;
                state = st_long(state);
            } else {
                pos = opt[cur].back_prev;
                if (pos < kNumRepDistances) state = st_long(state);
                else state = st_match(state);
            }
            optimal_t *o = &opt[pos_prev];
            if (pos < kNumRepDistances) {
                if (pos == 0) { e->reps[0] = o->backs[0]; e->reps[1] = o->backs[1]; e->reps[2] = o->backs[2]; e->reps[3] = o->backs[3]; }
                else if (pos == 1) { e->reps[0] = o->backs[1]; e->reps[1] = o->backs[0]; e->reps[2] = o->backs[2]; e->reps[3] = o->backs[3]; }
                else if (pos == 2) { e->reps[0] = o->backs[2]; e->reps[1] = o->backs[0]; e->reps[2] = o->backs[1]; e->reps[3] = o->backs[3]; }
                else { e->reps[0] = o->backs[3]; e->reps[1] = o->backs[0]; e->reps[2] = o->backs[1]; e->reps[3] = o->backs[2]; }
            } else {
                e->reps[0] = (uint32_t)(pos - kNumRepDistances);
                e->reps[1] = o->backs[0]; e->reps[2] = o->backs[1]; e->reps[3] = o->backs[2];
            }
        }
        opt[cur].state = state;
        for (i = 0; i < 4; i++) opt[cur].backs[i] = (int32_t)e->reps[i];
        uint32_t cur_price = opt[cur].price;
        cur_byte = bt_byte(&e->bt, -1);
        match_byte = bt_byte(&e->bt, (int32_t)(0 - e->reps[0] - 1 - 1));
        pos_state = position & e->pos_state_mask;
        uint32_t cur_and1_price = cur_price + price0(e->is_match[(state << kNumPosStatesBitsMax) + pos_state]) +
            lit_price(lit_coder(e, position, bt_byte(&e->bt, -2)), !st_is_char(state), match_byte, cur_byte);
        optimal_t *next = &opt[cur + 1];
        int next_is_char = 0;
        if (cur_and1_price < next->price) {
            next->price = cur_and1_price; next->pos_prev = (int32_t)cur; make_as_char(next); next_is_char = 1;
        }
        match_price = cur_price + price1(e->is_match[(state << kNumPosStatesBitsMax) + pos_state]);
        rep_match_price = match_price + price1(e->is_rep[state]);
        if (match_byte == cur_byte && !(next->pos_prev < (int32_t)cur && next->back_prev == 0)) {
            uint32_t short_rep_price = rep_match_price + get_rep_len1_price(e, state, pos_state);
            if (short_rep_price <= next->price) {
                next->price = short_rep_price; next->pos_prev = (int32_t)cur; make_as_short_rep(next); next_is_char = 1;
            }
        }
        uint32_t num_avail_full = bt_avail(&e->bt) + 1;
        if (kNumOpts - 1 - cur < num_avail_full) num_avail_full = kNumOpts - 1 - cur;
        num_avail = num_avail_full;
        if (num_avail < 2) continue;
        if (num_avail > e->num_fast_bytes) num_avail = e->num_fast_bytes;
        if (!next_is_char && match_byte != cur_byte) {
            /* Literal + rep0 */
            uint32_t t = num_avail_full - 1 < e->num_fast_bytes ? num_avail_full - 1 : e->num_fast_bytes;
            uint32_t len_test2 = bt_match_len(&e->bt, 0, e->reps[0], (int32_t)t);
            if (len_test2 >= 2) {
                uint32_t state2 = st_lit(state);
                uint32_t ps_next = (position + 1) & e->pos_state_mask;
                uint32_t next_rep_match_price = cur_and1_price +
                    price1(e->is_match[(state2 << kNumPosStatesBitsMax) + ps_next]) + price1(e->is_rep[state2]);
                uint32_t offset = cur + 1 + len_test2;
                while (len_end < offset) opt[++len_end].price = kIfinityPrice;
                uint32_t cl = next_rep_match_price + get_rep_price(e, 0, len_test2, state2, ps_next);
                optimal_t *o = &opt[offset];
                if (cl < o->price) {
                    o->price = cl; o->pos_prev = (int32_t)cur + 1; o->back_prev = 0; o->prev1_is_char = 1; o->prev2 = 0;
                }
            }
        }
        uint32_t start_len = 2;
        for (uint32_t ri = 0; ri < kNumRepDistances; ri++) {
            uint32_t len_test = bt_match_len(&e->bt, -1, e->reps[ri], (int32_t)num_avail);
            if (len_test < 2) continue;
            uint32_t len_test_tmp = len_test;
            do {
                while (len_end < cur + len_test) opt[++len_end].price = kIfinityPrice;
                uint32_t cl = rep_match_price + get_rep_price(e, ri, len_test, state, pos_state);
                optimal_t *o = &opt[cur + len_test];
                if (cl < o->price) { o->price = cl; o->pos_prev = (int32_t)cur; o->back_prev = (int32_t)ri; o->prev1_is_char = 0; }
            } while (--len_test >= 2);
            len_test = len_test_tmp;
            if (ri == 0) start_len = len_test + 1;
            if (len_test < num_avail_full) {
                uint32_t t = num_avail_full - 1 - len_test;
                if (t > e->num_fast_bytes) t = e->num_fast_bytes;
                uint32_t len_test2 = bt_match_len(&e->bt, (int32_t)len_test, e->reps[ri], (int32_t)t);
                if (len_test2 >= 2) {
                    uint32_t state2 = st_long(state);
                    uint32_t ps_next = (position + len_test) & e->pos_state_mask;
                    uint32_t cur_and_len_char_price = rep_match_price + get_rep_price(e, ri, len_test, state, pos_state) +
                        price0(e->is_match[(state2 << kNumPosStatesBitsMax) + ps_next]) +
                        lit_price(lit_coder(e, position + len_test, bt_byte(&e->bt, (int32_t)len_test - 1 - 1)), 1,
                                  bt_byte(&e->bt, (int32_t)len_test - 1 - (int32_t)(e->reps[ri] + 1)),
                                  bt_byte(&e->bt, (int32_t)len_test - 1));
                    state2 = st_lit(state2);
                    ps_next = (position + len_test + 1) & e->pos_state_mask;
                    uint32_t next_match_price = cur_and_len_char_price + price1(e->is_match[(state2 << kNumPosStatesBitsMax) + ps_next]);
                    uint32_t next_rep_match_price = next_match_price + price1(e->is_rep[state2]);
                    uint32_t offset = len_test + 1 + len_test2;
                    while (len_end < cur + offset) opt[++len_end].price = kIfinityPrice;
                    uint32_t cl = next_rep_match_price + get_rep_price(e, 0, len_test2, state2, ps_next);
                    optimal_t *o = &opt[cur + offset];
                    if (cl < o->price) {
                        o->price = cl; o->pos_prev = (int32_t)(cur + len_test + 1); o->back_prev = 0;
                        o->prev1_is_char = 1; o->prev2 = 1; o->pos_prev2 = (int32_t)cur; o->back_prev2 = (int32_t)ri;
                    }
                }
            }
        }
        if (new_len > num_avail) {
            new_len = num_avail;
            for (num_distance_pairs = 0; new_len > e->md_len[num_distance_pairs]; num_distance_pairs++) {}
            e->md_len[num_distance_pairs] = new_len;
            num_distance_pairs++;
        }
        if (new_len >= start_len) {
            normal_match_price = match_price + price0(e->is_rep[state]);
            while (len_end < cur + new_len) opt[++len_end].price = kIfinityPrice;
            uint32_t offs = 0;
            while (start_len > e->md_len[offs]) offs++;
            for (uint32_t len_test = start_len;; len_test++) {
                uint32_t cur_back = e->md_dist[offs];
                uint32_t cl = normal_match_price + get_pos_len_price(e, cur_back, len_test, pos_state);
                optimal_t *o = &opt[cur + len_test];
                if (cl < o->price) { o->price = cl; o->pos_prev = (int32_t)cur; o->back_prev = (int32_t)(cur_back + kNumRepDistances); o->prev1_is_char = 0; }
                if (len_test == e->md_len[offs]) {
                    if (len_test < num_avail_full) {
                        uint32_t t = num_avail_full - 1 - len_test;
                        if (t > e->num_fast_bytes) t = e->num_fast_bytes;
                        uint32_t len_test2 = bt_match_len(&e->bt, (int32_t)len_test, cur_back, (int32_t)t);
                        if (len_test2 >= 2) {
                            uint32_t state2 = st_match(state);
                            uint32_t ps_next = (position + len_test) & e->pos_state_mask;
                            uint32_t cur_and_len_char_price = cl +
                                price0(e->is_match[(state2 << kNumPosStatesBitsMax) + ps_next]) +
                                lit_price(lit_coder(e, position + len_test, bt_byte(&e->bt, (int32_t)len_test - 1 - 1)), 1,
                                          bt_byte(&e->bt, (int32_t)len_test - (int32_t)(cur_back + 1) - 1),
                                          bt_byte(&e->bt, (int32_t)len_test - 1));
                            state2 = st_lit(state2);
                            ps_next = (position + len_test + 1) & e->pos_state_mask;
                            uint32_t next_match_price = cur_and_len_char_price + price1(e->is_match[(state2 << kNumPosStatesBitsMax) + ps_next]);
                            uint32_t next_rep_match_price = next_match_price + price1(e->is_rep[state2]);
                            uint32_t offset = len_test + 1 + len_test2;
                            while (len_end < cur + offset) opt[++len_end].price = kIfinityPrice;
                            cl = next_rep_match_price + get_rep_price(e, 0, len_test2, state2, ps_next);
                            o = &opt[cur + offset];
                            if (cl < o->price) {
                                o->price = cl; o->pos_prev = (int32_t)(cur + len_test + 1); o->back_prev = 0;
                                o->prev1_is_char = 1; o->prev2 = 1; o->pos_prev2 = (int32_t)cur;
                                o->back_prev2 = (int32_t)(cur_back + kNumRepDistances);
                            }
                        }
                    }
                    offs++;
                    if (offs == num_distance_pairs) break;
                }
            }
        }
    }
}

static void write_end_marker(enc_t *e, uint32_t pos_state) { /* Encoder.java:818-835 */
    if (!e->prm.eos) return;
    re_encode(&e->rc, e->is_match, (e->state << kNumPosStatesBitsMax) + pos_state, 1);
    re_encode(&e->rc, e->is_rep, e->state, 0);
    e->state = st_match(e->state);
    uint32_t len = kMatchMinLen;
    len_encode(&e->len_enc, &e->rc, len - kMatchMinLen, pos_state);
    uint32_t pos_slot = (1u << kNumPosSlotBits) - 1;
    bt_enc(&e->rc, e->pos_slot[len_to_pos_state(len)], kNumPosSlotBits, pos_slot);
    uint32_t footer_bits = 30, pos_reduced = (1u << footer_bits) - 1;
    re_direct_bits(&e->rc, pos_reduced >> kNumAlignBits, (int)(footer_bits - kNumAlignBits));
    bt_rev_enc(&e->rc, e->pos_align, kNumAlignBits, pos_reduced & kAlignMask);
}
static void flush_enc(enc_t *e, uint32_t now_pos) { /* Encoder.java:837-841 */
    write_end_marker(e, now_pos & e->pos_state_mask);
    re_flush(&e->rc);
}

static void encode_rep(enc_t *e, int32_t pos, uint32_t len, uint32_t pos_state, uint32_t complex_state) { /* :938-974 */
    re_encode(&e->rc, e->is_rep, e->state, 1);
    if (pos == 0) {
        re_encode(&e->rc, e->is_rep_g0, e->state, 0);
        re_encode(&e->rc, e->is_rep0_long, complex_state, len == 1 ? 0 : 1);
    } else {
        re_encode(&e->rc, e->is_rep_g0, e->state, 1);
        if (pos == 1) re_encode(&e->rc, e->is_rep_g1, e->state, 0);
        else { re_encode(&e->rc, e->is_rep_g1, e->state, 1); re_encode(&e->rc, e->is_rep_g2, e->state, (uint32_t)pos - 2); }
    }
    if (len == 1) e->state = st_short(e->state);
    else { len_encode(&e->rep_len_enc, &e->rc, len - kMatchMinLen, pos_state); e->state = st_long(e->state); }
    uint32_t distance = e->rep_distances[pos];
    if (pos != 0) {
        for (int k = pos; k >= 1; k--) e->rep_distances[k] = e->rep_distances[k - 1];
        e->rep_distances[0] = distance;
    }
}
static void encode_match(enc_t *e, int32_t backp, uint32_t len, uint32_t pos_state) { /* :976-1005 */
    re_encode(&e->rc, e->is_rep, e->state, 0);
    e->state = st_match(e->state);
    len_encode(&e->len_enc, &e->rc, len - kMatchMinLen, pos_state);
    uint32_t pos = (uint32_t)(backp - kNumRepDistances);
    uint32_t pos_slot = get_pos_slot(pos);
    bt_enc(&e->rc, e->pos_slot[len_to_pos_state(len)], kNumPosSlotBits, pos_slot);
    if (pos_slot >= kStartPosModelIndex) {
        uint32_t footer_bits = (pos_slot >> 1) - 1;
        uint32_t base = (2 | (pos_slot & 1)) << footer_bits;
        uint32_t pos_reduced = pos - base;
        if (pos_slot < kEndPosModelIndex) rev_enc_at(&e->rc, e->pos_encoders, (int)(base - pos_slot - 1), (int)footer_bits, pos_reduced);
        else {
            re_direct_bits(&e->rc, pos_reduced >> kNumAlignBits, (int)(footer_bits - kNumAlignBits));
            bt_rev_enc(&e->rc, e->pos_align, kNumAlignBits, pos_reduced & kAlignMask);
            e->align_price_count++;
        }
    }
    e->rep_distances[3] = e->rep_distances[2]; e->rep_distances[2] = e->rep_distances[1];
    e->rep_distances[1] = e->rep_distances[0]; e->rep_distances[0] = pos;
    e->match_price_count++;
}

static int enc_run(enc_t *e, const uint8_t *in, uint64_t n) {
    const oracle_params *p = &e->prm;
    /* setters (Encoder.java:1135-1180) */
    uint32_t dict = (uint32_t)p->dict_size;
    uint32_t dls = 0;
    while (dict > (1u << dls)) dls++;
    e->dist_table_size = dls * 2;
    e->num_fast_bytes = (uint32_t)p->fb;
    e->lc = (uint32_t)p->lc; e->lp = (uint32_t)p->lp;
    e->pos_state_bits = (uint32_t)p->pb; e->pos_state_mask = (1u << p->pb) - 1;
    /* Create (Encoder.java:224-241) */
    if (bt_create(&e->bt, in, n, dict, e->num_fast_bytes, p->mf == 0 ? 2 : 4) != 0) return -2;
    size_t nlit = (size_t)1 << (e->lc + e->lp);
    if (!e->lit) e->lit = (uint16_t *)malloc(nlit * 0x300 * sizeof(uint16_t));
    if (!e->lit) return -2;
    e->out.n = 0; e->out.oom = 0;
    /* Init (Encoder.java:247-273) */
    e->state = 0; e->previous_byte = 0;
    for (int i = 0; i < 4; i++) e->rep_distances[i] = 0;
    e->rc.out = &e->out;
    re_init(&e->rc);
    init_probs(e->is_match, sizeof(e->is_match) / 2);
    init_probs(e->is_rep, kNumStates); init_probs(e->is_rep_g0, kNumStates);
    init_probs(e->is_rep_g1, kNumStates); init_probs(e->is_rep_g2, kNumStates);
    init_probs(e->is_rep0_long, sizeof(e->is_rep0_long) / 2);
    init_probs(e->pos_encoders, sizeof(e->pos_encoders) / 2);
    init_probs(e->lit, nlit * 0x300);
    for (int i = 0; i < kNumLenToPosStates; i++) init_probs(e->pos_slot[i], 1 << kNumPosSlotBits);
    len_init(&e->len_enc, 1u << e->pos_state_bits);
    len_init(&e->rep_len_enc, 1u << e->pos_state_bits);
    init_probs(e->pos_align, 1 << kNumAlignBits);
    e->longest_match_found = 0; e->optimum_end = 0; e->optimum_cur = 0; e->additional_offset = 0;
    /* SetStreams (Encoder.java:1046-1062) */
    fill_distances_prices(e);
    fill_align_prices(e);
    e->len_enc.table_size = e->num_fast_bytes + 1 - kMatchMinLen;
    for (uint32_t ps = 0; ps < (1u << e->pos_state_bits); ps++) len_update_table(&e->len_enc, ps);
    e->rep_len_enc.table_size = e->num_fast_bytes + 1 - kMatchMinLen;
    for (uint32_t ps = 0; ps < (1u << e->pos_state_bits); ps++) len_update_table(&e->rep_len_enc, ps);

    /* CodeOneBlock / encodeOne (Encoder.java:843-936), progress blocks folded */
    uint64_t now_pos = 0;
    if (bt_avail(&e->bt) == 0) { flush_enc(e, 0); return e->out.oom ? -2 : 0; }
    read_match_distances(e);
    {
        uint32_t ps = (uint32_t)now_pos & e->pos_state_mask;
        re_encode(&e->rc, e->is_match, (e->state << kNumPosStatesBitsMax) + ps, 0);
        e->state = st_lit(e->state);
        uint8_t cb = bt_byte(&e->bt, 0 - e->additional_offset);
        lit_encode(&e->rc, lit_coder(e, (uint32_t)now_pos, e->previous_byte), cb);
        e->previous_byte = cb;
        e->additional_offset--;
        now_pos++;
    }
    if (bt_avail(&e->bt) == 0) { flush_enc(e, (uint32_t)now_pos); return e->out.oom ? -2 : 0; }
    for (;;) {
        int32_t back;
        uint32_t len = get_optimum(e, (uint32_t)now_pos, &back);
        uint32_t ps = (uint32_t)now_pos & e->pos_state_mask;
        uint32_t cs = (e->state << kNumPosStatesBitsMax) + ps;
        if (len == 1 && back == -1) {
            re_encode(&e->rc, e->is_match, cs, 0);
            /* encodeSingleByteLiteral (Encoder.java:1007-1024) */
            uint8_t cb = bt_byte(&e->bt, 0 - e->additional_offset);
            uint16_t *sub = lit_coder(e, (uint32_t)now_pos, e->previous_byte);
            if (st_is_char(e->state)) lit_encode(&e->rc, sub, cb);
            else {
                uint8_t mb = bt_byte(&e->bt, (int32_t)(0 - e->rep_distances[0] - 1) - e->additional_offset);
                lit_encode_matched(&e->rc, sub, mb, cb);
            }
            e->previous_byte = cb;
            e->state = st_lit(e->state);
        } else {
            re_encode(&e->rc, e->is_match, cs, 1);
            if (back < kNumRepDistances) encode_rep(e, back, len, ps, cs);
            else encode_match(e, back, len, ps);
            e->previous_byte = bt_byte(&e->bt, (int32_t)len - 1 - e->additional_offset);
        }
        e->additional_offset -= (int32_t)len;
        now_pos += len;
        if (e->additional_offset == 0) {
            if (e->match_price_count >= (1u << 7)) fill_distances_prices(e);
            if (e->align_price_count >= kAlignTableSize) fill_align_prices(e);
            if (bt_avail(&e->bt) == 0) { flush_enc(e, (uint32_t)now_pos); break; }
        }
    }
    return e->out.oom ? -2 : 0;
}

void oracle_write_props(const oracle_params *p, uint8_t out[5]) {
    out[0] = (uint8_t)((p->pb * 5 + p->lp) * 9 + p->lc);
    for (int i = 0; i < 4; i++) out[1 + i] = (uint8_t)((uint32_t)p->dict_size >> (8 * i));
}

static int check_params(const oracle_params *p) {
    if (p->dict_size < 1 || p->dict_size > (1 << 29)) return -1;
    if (p->fb < 5 || p->fb > kMatchMaxLen) return -1;
    if (p->mf < 0 || p->mf > 2) return -1;
    if (p->lp < 0 || p->lp > 4 || p->lc < 0 || p->lc > 8 || p->pb < 0 || p->pb > 4) return -1;
    return 0;
}

int64_t oracle_match_lists(const uint8_t *in, uint64_t n, const oracle_params *p,
                           uint32_t *counts, uint32_t *main_len,
                           uint32_t *lens, uint32_t *dists, uint64_t cap) {
    init_tables();
    if (check_params(p) != 0) return -1;
    bt_t t;
    memset(&t, 0, sizeof t);
    if (bt_create(&t, in, n, (uint32_t)p->dict_size, (uint32_t)p->fb, p->mf == 0 ? 2 : 4) != 0) { bt_free(&t); return -1; }
    uint32_t l[kMatchMaxLen + 1], d[kMatchMaxLen + 1];
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) {
        uint32_t c = bt_get_matches(&t, l, d);
        counts[i] = c;
        uint32_t ml = 0;
        if (c > 0) {
            ml = l[c - 1];
            if (ml == (uint32_t)p->fb) ml += bt_match_len(&t, (int32_t)ml - 1, d[c - 1], (int32_t)(kMatchMaxLen - ml));
        }
        main_len[i] = ml;
        if (total + c > cap) { bt_free(&t); return -1; }
        for (uint32_t k = 0; k < c; k++) { lens[total + k] = l[k]; dists[total + k] = d[k]; }
        total += c;
    }
    bt_free(&t);
    return (int64_t)total;
}

int oracle_encode(const uint8_t *in, uint64_t n, const oracle_params *p, int mode,
                  uint8_t **out, uint64_t *out_len) {
    init_tables();
    if (check_params(p) != 0) return -1;
    enc_t *e = (enc_t *)calloc(1, sizeof(enc_t));
    if (!e) return -2;
    e->prm = *p;
    e->mode = mode;
    uint32_t *cnt = NULL, *ml = NULL, *pl = NULL, *pd = NULL;
    uint64_t *offs = NULL;
    int rc = 0;
    if (mode == 1) {
        uint64_t cap = n * 8 + 16;
        cnt = (uint32_t *)malloc((n + 1) * 4); ml = (uint32_t *)malloc((n + 1) * 4);
        offs = (uint64_t *)malloc((n + 1) * 8);
        for (;;) {
            pl = (uint32_t *)malloc(cap * 4); pd = (uint32_t *)malloc(cap * 4);
            if (!cnt || !ml || !offs || !pl || !pd) { rc = -2; goto done; }
            int64_t tot = oracle_match_lists(in, n, p, cnt, ml, pl, pd, cap);
            if (tot >= 0) break;
            free(pl); free(pd); pl = pd = NULL;
            cap *= 4;
        }
        uint64_t o = 0;
        for (uint64_t i = 0; i < n; i++) { offs[i] = o; o += cnt[i]; }
        e->pre_counts = cnt; e->pre_main = ml; e->pre_lens = pl; e->pre_dists = pd; e->pre_offs = offs;
    }
    rc = enc_run(e, in, n);
    if (rc == 0) { *out = e->out.p; *out_len = e->out.n; e->out.p = NULL; }
done:
    free(e->out.p);
    free(e->lit);
    bt_free(&e->bt);
    free(cnt); free(ml); free(pl); free(pd); free(offs);
    free(e);
    return rc;
}

void oracle_free(void *ptr) { free(ptr); }

/* A session = one reused Encoder instance (one instance per
 * thread, as a Java caller keeps one Encoder and calls Code per chunk). */
struct oracle_enc { enc_t *e; };

oracle_enc *oracle_enc_new(const oracle_params *p) {
    init_tables();
    if (check_params(p) != 0) return NULL;
    oracle_enc *s = (oracle_enc *)calloc(1, sizeof(oracle_enc));
    if (!s) return NULL;
    s->e = (enc_t *)calloc(1, sizeof(enc_t));
    if (!s->e) { free(s); return NULL; }
    s->e->prm = *p;
    return s;
}

int oracle_enc_code(oracle_enc *s, const uint8_t *in, uint64_t n, const uint8_t **out, uint64_t *out_len) {
    enc_t *e = s->e;
    /* reset the per-call state the way Encoder.Init/SetStreams do; keep the buffers */
    bt_t bt = e->bt;
    uint16_t *lit = e->lit;
    obuf_t ob = e->out;
    oracle_params prm = e->prm;
    memset(e, 0, sizeof(*e));
    e->bt = bt; e->lit = lit; e->out = ob; e->prm = prm;
    int rc = enc_run(e, in, n);
    if (rc != 0) return rc;
    *out = e->out.p;
    *out_len = e->out.n;
    return 0;
}

void oracle_enc_delete(oracle_enc *s) {
    if (!s) return;
    free(s->e->out.p);
    free(s->e->lit);
    bt_free(&s->e->bt);
    free(s->e);
    free(s);
}

/* ============================================================ decoder */
typedef struct {
    const uint8_t *in; uint64_t n, pos;
    uint32_t range, code;
} rdec_t;

static inline uint32_t rd_read(rdec_t *d) { /* InputStream.read(): -1 at EOF */
    return d->pos < d->n ? d->in[d->pos++] : 0xFFFFFFFFu;
}
static void rd_init(rdec_t *d) { /* RangeDecoder.java:19-25 */
    d->code = 0; d->range = 0xFFFFFFFFu;
    for (int i = 0; i < 5; i++) d->code = (d->code << 8) | rd_read(d);
}
static uint32_t rd_direct(rdec_t *d, int nbits) { /* RangeDecoder.java:27-41 */
    uint32_t result = 0;
    for (int i = nbits; i != 0; i--) {
        d->range >>= 1;
        uint32_t t = (d->code - d->range) >> 31;
        d->code -= d->range & (t - 1);
        result = (result << 1) | (1 - t);
        if ((d->range & kTopMask) == 0) { d->code = (d->code << 8) | rd_read(d); d->range <<= 8; }
    }
    return result;
}
static uint32_t rd_bit(rdec_t *d, uint16_t *probs, uint32_t idx) { /* RangeDecoder.java:43-64 */
    uint32_t prob = probs[idx];
    uint32_t bound = (d->range >> 11) * prob;
    if (d->code < bound) {   /* (code ^ 0x80000000) < (bound ^ 0x80000000): unsigned compare */
        d->range = bound;
        probs[idx] = (uint16_t)(prob + ((kBitModelTotal - prob) >> kNumMoveBits));
        if ((d->range & kTopMask) == 0) { d->code = (d->code << 8) | rd_read(d); d->range <<= 8; }
        return 0;
    }
    d->range -= bound; d->code -= bound;
    probs[idx] = (uint16_t)(prob - (prob >> kNumMoveBits));
    if ((d->range & kTopMask) == 0) { d->code = (d->code << 8) | rd_read(d); d->range <<= 8; }
    return 1;
}
static uint32_t bt_dec(rdec_t *d, uint16_t *probs, int nbits) { /* BitTreeDecoder.java:19-25 */
    uint32_t m = 1;
    for (int b = nbits; b != 0; b--) m = (m << 1) + rd_bit(d, probs, m);
    return m - (1u << nbits);
}
static uint32_t bt_rev_dec(rdec_t *d, uint16_t *probs, int nbits) { /* BitTreeDecoder.java:27-37 */
    uint32_t m = 1, sym = 0;
    for (int b = 0; b < nbits; b++) { uint32_t bit = rd_bit(d, probs, m); m <<= 1; m += bit; sym |= bit << b; }
    return sym;
}
static uint32_t rev_dec_at(rdec_t *d, uint16_t *models, int start, int nbits) { /* Decoder.java:13-23 */
    uint32_t m = 1, sym = 0;
    for (int b = 0; b < nbits; b++) { uint32_t bit = rd_bit(d, models, start + m); m <<= 1; m += bit; sym |= bit << b; }
    return sym;
}
typedef struct { uint16_t choice[2], low[16][8], mid[16][8], high[256]; } lendec_t;
static uint32_t len_dec(rdec_t *d, lendec_t *l, uint32_t ps) { /* Decoder.java:48-59 */
    if (rd_bit(d, l->choice, 0) == 0) return bt_dec(d, l->low[ps], 3);
    uint32_t sym = kNumLowLenSymbols;
    if (rd_bit(d, l->choice, 1) == 0) sym += bt_dec(d, l->mid[ps], 3);
    else sym += kNumMidLenSymbols + bt_dec(d, l->high, 8);
    return sym;
}

int oracle_decode(const uint8_t *in, uint64_t n_in, const uint8_t props[5], int64_t out_size,
                  uint8_t *out, uint64_t out_cap, uint64_t *out_len) {
    init_tables();
    /* SetDecoderProperties (Decoder.java:303-318) */
    uint32_t val = props[0];
    uint32_t lc = val % 9, rem = val / 9, lp = rem % 5, pb = rem / 5;
    uint32_t dict = 0;
    for (int i = 0; i < 4; i++) dict += (uint32_t)props[1 + i] << (i * 8);
    if (lc > 8 || lp > 4 || pb > 4) return -1;
    if ((int32_t)dict < 0) return -1;                 /* SetDictionarySize :160-170 */
    uint32_t dict_check = dict > 1 ? dict : 1;
    uint16_t is_match[192], is_rep[12], g0[12], g1[12], g2[12], rep0_long[192];
    uint16_t pos_slot[4][64], pos_dec[114], align[16];
    lendec_t len_d, rep_len_d;
    size_t nlit = (size_t)1 << (lc + lp);
    uint16_t *lit = (uint16_t *)malloc(nlit * 0x300 * 2);
    if (!lit) return -1;
    /* Init (Decoder.java:184-203) */
    init_probs(is_match, 192); init_probs(rep0_long, 192); init_probs(is_rep, 12);
    init_probs(g0, 12); init_probs(g1, 12); init_probs(g2, 12); init_probs(pos_dec, 114);
    init_probs(lit, nlit * 0x300);
    for (int i = 0; i < 4; i++) init_probs(pos_slot[i], 64);
    init_probs((uint16_t *)&len_d, sizeof(len_d) / 2);
    init_probs((uint16_t *)&rep_len_d, sizeof(rep_len_d) / 2);
    init_probs(align, 16);
    rdec_t d = { in, n_in, 0, 0, 0 };
    rd_init(&d);
    uint32_t pos_mask = (1u << pb) - 1;
    uint32_t state = 0, rep0 = 0, rep1 = 0, rep2 = 0, rep3 = 0;
    uint64_t now = 0;
    uint8_t prev = 0;
    int ok = 1;
    /* Code (Decoder.java:205-301) */
    while (out_size < 0 || (int64_t)now < out_size) {
        uint32_t ps = (uint32_t)now & pos_mask;
        if (rd_bit(&d, is_match, (state << 4) + ps) == 0) {
            uint16_t *sub = lit + (size_t)((((uint32_t)now & ((1u << lp) - 1)) << lc) + ((uint32_t)prev >> (8 - lc))) * 0x300;
            uint32_t sym = 1;
            if (st_is_char(state)) {
                do { sym = (sym << 1) | rd_bit(&d, sub, sym); } while (sym < 0x100);
            } else {
                uint32_t mb = out[now - rep0 - 1];
                do {
                    uint32_t mbit = (mb >> 7) & 1; mb <<= 1;
                    uint32_t bit = rd_bit(&d, sub, ((1 + mbit) << 8) + sym);
                    sym = (sym << 1) | bit;
                    if (mbit != bit) { while (sym < 0x100) sym = (sym << 1) | rd_bit(&d, sub, sym); break; }
                } while (sym < 0x100);
            }
            prev = (uint8_t)sym;
            if (now >= out_cap) { ok = -1; break; }
            out[now++] = prev;
            state = st_lit(state);
        } else {
            uint32_t len;
            if (rd_bit(&d, is_rep, state) == 1) {
                len = 0;
                if (rd_bit(&d, g0, state) == 0) {
                    if (rd_bit(&d, rep0_long, (state << 4) + ps) == 0) { state = st_short(state); len = 1; }
                } else {
                    uint32_t dist;
                    if (rd_bit(&d, g1, state) == 0) dist = rep1;
                    else {
                        if (rd_bit(&d, g2, state) == 0) dist = rep2;
                        else { dist = rep3; rep3 = rep2; }
                        rep2 = rep1;
                    }
                    rep1 = rep0; rep0 = dist;
                }
                if (len == 0) { len = len_dec(&d, &rep_len_d, ps) + kMatchMinLen; state = st_long(state); }
            } else {
                rep3 = rep2; rep2 = rep1; rep1 = rep0;
                len = kMatchMinLen + len_dec(&d, &len_d, ps);
                state = st_match(state);
                uint32_t slot = bt_dec(&d, pos_slot[len_to_pos_state(len)], 6);
                if (slot >= kStartPosModelIndex) {
                    uint32_t ndb = (slot >> 1) - 1;
                    rep0 = (2 | (slot & 1)) << ndb;
                    if (slot < kEndPosModelIndex) rep0 += rev_dec_at(&d, pos_dec, (int)(rep0 - slot - 1), (int)ndb);
                    else {
                        rep0 += rd_direct(&d, (int)(ndb - kNumAlignBits)) << kNumAlignBits;
                        rep0 += bt_rev_dec(&d, align, kNumAlignBits);
                        if ((int32_t)rep0 < 0) {
                            if (rep0 == 0xFFFFFFFFu) break;   /* end marker */
                            ok = 0; break;
                        }
                    }
                } else rep0 = slot;
            }
            if ((uint64_t)rep0 >= now || rep0 >= dict_check) { ok = 0; break; }
            /* OutWindow.CopyBlock (OutWindow.java:53-67) */
            for (uint32_t k = 0; k < len; k++) {
                if (now >= out_cap) { ok = -1; break; }
                out[now] = out[now - rep0 - 1];
                now++;
            }
            if (ok != 1) break;
            prev = out[now - 1];
        }
    }
    free(lit);
    *out_len = now;
    return ok;
}

/* ---------------------------------------------------- unit test hooks */
int oracle_rc_encode_bits(const int32_t *bits, int n, uint8_t *out, int cap) {
    init_tables();
    obuf_t ob = { 0 };
    renc_t r; r.out = &ob; re_init(&r);
    uint16_t probs[kNumStates]; init_probs(probs, kNumStates);
    for (int i = 0; i < n; i++) re_encode(&r, probs, 4, (uint32_t)bits[i]);
    re_flush(&r);
    int len = (int)ob.n;
    if (len > cap) len = -1; else memcpy(out, ob.p, ob.n);
    free(ob.p);
    return len;
}
int oracle_rc_direct_bits(const uint32_t *vals, const int32_t *nbits, int n, uint8_t *out, int cap) {
    init_tables();
    obuf_t ob = { 0 };
    renc_t r; r.out = &ob; re_init(&r);
    for (int i = 0; i < n; i++) re_direct_bits(&r, vals[i], nbits[i]);
    re_flush(&r);
    int len = (int)ob.n;
    if (len > cap) len = -1; else memcpy(out, ob.p, ob.n);
    free(ob.p);
    return len;
}
void oracle_bittree_prices_after(int nbits, int sym, uint32_t *prices) {
    init_tables();
    obuf_t ob = { 0 };
    renc_t r; r.out = &ob; re_init(&r);
    uint16_t probs[1 << 8]; init_probs(probs, (size_t)1 << nbits);
    bt_enc(&r, probs, nbits, (uint32_t)sym);
    for (int s = 0; s < (1 << nbits); s++) prices[s] = bt_price(probs, nbits, (uint32_t)s);
    free(ob.p);
}
