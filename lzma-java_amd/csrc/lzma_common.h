// lzma_common.h -- shared constants, parameter derivation and lookup tables
// for the MI355X LZMA path. All constants restate
// src/main/java/SevenZip/Compression/LZMA/Base.java and the RangeCoder
// classes of rfalke/lzma-java; cited per item.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/lzma_mi355x.h"

// Lanes per wavefront. gfx950 runs wave64; the per-stream kernels (enc, dec)
// are one wavefront per workgroup and size every lane loop by kWave. The only
// other value ever used is 1, by the CPU emulation build in tests/simt.
#ifndef LZG_WAVE
#define LZG_WAVE 64
#endif

namespace lzg {

constexpr int kWave = LZG_WAVE;
constexpr int kNumOpts = 1 << 12;               // Encoder.java:19
constexpr uint32_t kInfinityPrice = 0xFFFFFFF;  // Encoder.java:22
constexpr int kNumRepDistances = 4;             // Base.java:4
constexpr int kNumStates = 12;                  // Base.java:5
constexpr int kNumPosSlotBits = 6;              // Base.java:42
constexpr int kNumLenToPosStates = 4;           // Base.java:48
constexpr int kMatchMinLen = 2;                 // Base.java:50
constexpr int kNumAlignBits = 4;                // Base.java:60
constexpr int kAlignTableSize = 16;
constexpr int kAlignMask = 15;
constexpr int kStartPosModelIndex = 4;          // Base.java:64
constexpr int kEndPosModelIndex = 14;
constexpr int kNumFullDistances = 128;          // Base.java:68
constexpr int kNumPosStatesBitsMax = 4;         // Base.java:73
constexpr int kNumPosStatesMax = 16;
constexpr int kNumLowLenSymbols = 8;            // Base.java:78-84
constexpr int kNumMidLenSymbols = 8;
constexpr int kNumLenSymbols = 272;
constexpr int kMatchMaxLen = 273;               // Base.java:85
constexpr uint32_t kBitModelTotal = 2048;       // RangeBase.java:5
constexpr int kNumMoveBits = 5;                 // RangeBase.java:7
constexpr uint32_t kTopMask = 0xFF000000u;      // RangeBase.java:6
constexpr uint32_t kNoPos = 0xFFFFFFFFu;

// Probability-model layout of one stream (u16 each), shared by encoder and
// decoder kernels. Offsets in elements.
constexpr int P_IS_MATCH = 0;                          // 12 << 4
constexpr int P_IS_REP = P_IS_MATCH + 192;
constexpr int P_IS_REP_G0 = P_IS_REP + 12;
constexpr int P_IS_REP_G1 = P_IS_REP_G0 + 12;
constexpr int P_IS_REP_G2 = P_IS_REP_G1 + 12;
constexpr int P_IS_REP0_LONG = P_IS_REP_G2 + 12;      // 12 << 4
constexpr int P_POS_SLOT = P_IS_REP0_LONG + 192;      // 4 x 64
constexpr int P_POS_ENC = P_POS_SLOT + 256;           // 114 (kNumFullDistances - kEndPosModelIndex)
constexpr int P_ALIGN = P_POS_ENC + 114;              // 16
constexpr int P_LEN = P_ALIGN + 16;                   // len coder: choice 2, low 16x8, mid 16x8, high 256
constexpr int LEN_CHOICE = 0, LEN_LOW = 2, LEN_MID = 2 + 128, LEN_HIGH = 2 + 256, LEN_SIZE = 2 + 256 + 256;
constexpr int P_REP_LEN = P_LEN + LEN_SIZE;
constexpr int P_LIT = P_REP_LEN + LEN_SIZE;           // literal coders follow (may live elsewhere)
constexpr int P_FIXED_COUNT = P_LIT;                  // 1852 u16

// Probability layout used by the encoder and decoder kernels (the models of
// Encoder.java:113-128 / Decoder.java:138-152). The
// posState-indexed models (isMatch, isRep0Long, the low/mid length coders) are
// strided by 1 << PBS posStates: PBS = 2 serves pb <= 2 (the common case, and
// 1.3 KiB less LDS per stream than the 16-posState layout), PBS = 4 serves pb 3-4.
template <int PBS>
struct ProbLayout {
    static constexpr int IS_MATCH = 0;
    static constexpr int IS_REP = IS_MATCH + (kNumStates << PBS);
    static constexpr int G0 = IS_REP + kNumStates, G1 = G0 + kNumStates, G2 = G1 + kNumStates;
    static constexpr int R0L = G2 + kNumStates;
    static constexpr int PSLOT = R0L + (kNumStates << PBS);
    static constexpr int PENC = PSLOT + (kNumLenToPosStates << kNumPosSlotBits);
    static constexpr int ALIGN = PENC + (kNumFullDistances - kEndPosModelIndex);
    static constexpr int LOW = 2, MID = LOW + (8 << PBS), HIGH = MID + (8 << PBS), LSIZE = HIGH + 256;
    static constexpr int LEN = ALIGN + kAlignTableSize;
    static constexpr int RLEN = LEN + LSIZE;
    static constexpr int COUNT = RLEN + LSIZE;
};
__host__ __device__ constexpr uint32_t prob_count(uint32_t pb) {
    return pb <= 2 ? (uint32_t)ProbLayout<2>::COUNT : (uint32_t)ProbLayout<4>::COUNT;
}
// the decision models (isMatch, isRep, isRepG0-2, isRep0Long) are the first PSLOT entries
__host__ __device__ constexpr uint32_t dm_count(uint32_t pb) {
    return pb <= 2 ? (uint32_t)ProbLayout<2>::PSLOT : (uint32_t)ProbLayout<4>::PSLOT;
}


struct Tables {
    uint32_t crc[256];       // CRC.java:11-25 (also the BT4 hash mixer, BinTree.java:381)
    uint32_t prices[512];    // ProbPrices.java:8-18
    uint8_t fastpos[2048];   // Encoder.java:30-41
};

constexpr Tables make_tables() {
    Tables t{};
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t r = i;
        for (int j = 0; j < 8; j++) r = (r & 1) ? (r >> 1) ^ 0xEDB88320u : (r >> 1);
        t.crc[i] = r;
    }
    const int kNumBits = 9;
    for (int i = kNumBits - 1; i >= 0; i--) {
        uint32_t s = 1u << (kNumBits - i - 1), e = 1u << (kNumBits - i);
        for (uint32_t j = s; j < e; j++) t.prices[j] = ((uint32_t)i << 6) + (((e - j) << 6) >> (kNumBits - i - 1));
    }
    t.fastpos[0] = 0;
    t.fastpos[1] = 1;
    int c = 2;
    for (int slot = 2; slot < 22; slot++) {
        int k = 1 << ((slot >> 1) - 1);
        for (int j = 0; j < k; j++, c++) t.fastpos[c] = (uint8_t)slot;
    }
    return t;
}

// Fair wave priority for the one-stream-per-wave kernels. The sequencer issues
// oldest-first among waves of equal priority, so the first two waves of each
// SIMD run ahead and the last two finish alone at half occupancy (measured:
// profiles/r01_enc_placement.txt). Every `step` bytes a wave publishes its
// progress (fraction of its stream) in its CU's row of a per-kernel table,
// reads the row back and sets s_setprio by its rank on the CU: the slowest
// quarter gets priority 3, the fastest 0. Slots hold progress + 1, 0 = empty.
// Table rows: 2048 CUs (xcc, se, sh, cu of HW_ID / XCC_ID) x 64 waves (simd, wave).
constexpr uint32_t kSchedRows = 2048, kSchedCols = 64;
#if LZG_WAVE == 64 && !defined(LZG_NO_FAIRPRIO)
#define LZG_FAIRPRIO 1   // -DLZG_NO_FAIRPRIO: an experiment build without it
#else
#define LZG_FAIRPRIO 0
#endif
struct FairPrio {
    uint32_t* row;
    uint32_t slot, next, step;
    float scale;
    __device__ inline void start(uint32_t* table, uint32_t len, uint32_t lane) {
#if LZG_FAIRPRIO
        const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);           // HW_REG_HW_ID
        const uint32_t xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20) & 7u;   // HW_REG_XCC_ID
        const uint32_t cu = (((xcc * 8u + ((hw >> 13) & 7u)) * 2u + ((hw >> 12) & 1u)) * 16u) + ((hw >> 8) & 15u);
        row = table + (size_t)cu * kSchedCols;
        slot = ((hw >> 4) & 3u) * 16u + (hw & 15u);
        step = len >> 8 > 256u ? len >> 8 : 256u;
        next = step;
        scale = 65536.0f / (float)(len ? len : 1u);
        if (lane == 0) __hip_atomic_store(row + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_s_setprio(3);
#else
        (void)table; (void)len; (void)lane;
#endif
    }
    __device__ inline void update(uint32_t pos, uint32_t lane) {
#if LZG_FAIRPRIO
        if (pos < next) return;
        next = pos + step;
        const uint32_t prog = (uint32_t)((float)pos * scale) + 1u;
        if (lane == 0) __hip_atomic_store(row + slot, prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t v = __hip_atomic_load(row + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t nact = (uint32_t)__builtin_popcountll(__ballot(v != 0u));
        const uint32_t slower = (uint32_t)__builtin_popcountll(__ballot(v != 0u && v < prog));
        const uint32_t q = nact ? (slower * 4u) / nact : 0u;   // 0: among the slowest quarter
        switch (q) {
            case 0: __builtin_amdgcn_s_setprio(3); break;
            case 1: __builtin_amdgcn_s_setprio(2); break;
            case 2: __builtin_amdgcn_s_setprio(1); break;
            default: __builtin_amdgcn_s_setprio(0); break;
        }
#else
        (void)pos; (void)lane;
#endif
    }
    __device__ inline void finish(uint32_t lane) {
#if LZG_FAIRPRIO
        if (lane == 0) __hip_atomic_store(row + slot, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
        (void)lane;
#endif
    }
};

// Everything the kernels derive from lzma_params (Encoder.java:1135-1180,
// BinTree.java:59-134).
struct Derived {
    uint32_t dict_size, fb, lc, lp, pb, eos;
    uint32_t hash_array;          // BT4 (mf 1,2) vs BT2 (mf 0)
    uint32_t min_match_check;     // 4 / 3
    uint32_t direct_bytes;        // 0 / 2
    uint32_t hash_mask;           // BT4 hv mask (BinTree.java:115-129)
    uint32_t hash_bits;           // bits in hv (sort key width)
    uint32_t cut_value;           // 16 + fb/2 (BinTree.java:98)
    uint64_t cyc_size;            // dict + 1 (BinTree.java:107)
    uint32_t dist_table_size;     // 2*ceil(log2 dict) (Encoder.java:1141-1144)
    uint32_t pos_state_mask;
    uint32_t len_table_size;      // fb + 1 - 2 (Encoder.java:1058)
};

inline int derive(const lzma_params& p, Derived& d) {
    if (p.dict_size < 1 || p.dict_size > (1 << 29)) return LZMA_E_PARAM;
    if (p.fb < 5 || p.fb > kMatchMaxLen) return LZMA_E_PARAM;
    if (p.mf < 0 || p.mf > 2) return LZMA_E_PARAM;
    if (p.lc < 0 || p.lc > 8 || p.lp < 0 || p.lp > 4 || p.pb < 0 || p.pb > 4) return LZMA_E_PARAM;
    d.dict_size = (uint32_t)p.dict_size;
    d.fb = (uint32_t)p.fb;
    d.lc = (uint32_t)p.lc;
    d.lp = (uint32_t)p.lp;
    d.pb = (uint32_t)p.pb;
    d.eos = p.eos ? 1u : 0u;
    d.hash_array = p.mf != 0;
    d.min_match_check = d.hash_array ? 4 : 3;
    d.direct_bytes = d.hash_array ? 0 : 2;
    if (d.hash_array) {
        int32_t h = (int32_t)d.dict_size - 1;
        h |= (h >> 1); h |= (h >> 2); h |= (h >> 4); h |= (h >> 8);
        h >>= 1;
        h |= 0xFFFF;
        if (h > (1 << 24)) h >>= 1;
        d.hash_mask = (uint32_t)h;
    } else {
        d.hash_mask = 0xFFFF;
    }
    uint32_t hb = 0;
    while (hb < 32 && (d.hash_mask >> hb) != 0) hb++;
    d.hash_bits = hb;
    d.cut_value = 16 + (d.fb >> 1);
    d.cyc_size = (uint64_t)d.dict_size + 1;
    uint32_t dls = 0;
    while (d.dict_size > (1u << dls)) dls++;
    d.dist_table_size = dls * 2;
    d.pos_state_mask = (1u << d.pb) - 1;
    d.len_table_size = d.fb + 1 - kMatchMinLen;
    return LZMA_OK;
}

// Base.java:16-40 state machine.
__host__ __device__ inline uint32_t st_lit(uint32_t s) { return s < 4 ? 0 : (s < 10 ? s - 3 : s - 6); }
__host__ __device__ inline uint32_t st_match(uint32_t s) { return s < 7 ? 7 : 10; }
__host__ __device__ inline uint32_t st_short(uint32_t s) { return s < 7 ? 9 : 11; }
__host__ __device__ inline uint32_t st_long(uint32_t s) { return s < 7 ? 8 : 11; }
__host__ __device__ inline bool st_is_char(uint32_t s) { return s < 7; }
__host__ __device__ inline uint32_t len_to_pos_state(uint32_t len) { len -= kMatchMinLen; return len < 4 ? len : 3; }

// Match pair packing. u32: dist in 23 bits, len in 9 bits (streams <= 8 MiB);
// u64: dist in 32 bits, len above.
template <typename PairT> struct PairPack;
template <> struct PairPack<uint32_t> {
    static constexpr uint64_t kMaxStream = 1ull << 23;
    __device__ static inline uint32_t pack(uint32_t len, uint32_t dist) { return (len << 23) | dist; }
    __device__ static inline uint32_t len(uint32_t p) { return p >> 23; }
    __device__ static inline uint32_t dist(uint32_t p) { return p & 0x7FFFFFu; }
};
template <> struct PairPack<uint64_t> {
    static constexpr uint64_t kMaxStream = 1ull << 32;
    __device__ static inline uint64_t pack(uint32_t len, uint32_t dist) { return ((uint64_t)len << 32) | dist; }
    __device__ static inline uint32_t len(uint64_t p) { return (uint32_t)(p >> 32); }
    __device__ static inline uint32_t dist(uint64_t p) { return (uint32_t)p; }
};
constexpr int kInlinePairs = 4;

// Per-position match-list record (mf_walk writes it, the parser reads it): the
// first kInlinePairs pairs, then the info word (pair count | extended longest
// length << 16) in a vector of its own. One lane writes a whole record with
// 16-byte stores, so every 32-byte sector it touches is written in full (the
// u32 record is exactly one sector) -- no partial-sector write-back from L2.
typedef uint32_t v4u32 __attribute__((vector_size(16)));
template <typename PairT> constexpr uint32_t rec_vecs() { return (uint32_t)(sizeof(PairT) * kInlinePairs / 16 + 1); }
inline uint32_t rec_bytes(bool wide) { return 16u * (wide ? rec_vecs<uint64_t>() : rec_vecs<uint32_t>()); }

template <typename PairT>
__device__ inline void store_rec(v4u32* r, PairT q0, PairT q1, PairT q2, PairT q3, uint32_t info) {
    const v4u32 iv = {info, 0u, 0u, 0u};
    if constexpr (sizeof(PairT) == 4) {
        const v4u32 pv = {q0, q1, q2, q3};
        __builtin_nontemporal_store(pv, r + 0);
        __builtin_nontemporal_store(iv, r + 1);
    } else {
        const v4u32 pa = {(uint32_t)q0, (uint32_t)(q0 >> 32), (uint32_t)q1, (uint32_t)(q1 >> 32)};
        const v4u32 pb = {(uint32_t)q2, (uint32_t)(q2 >> 32), (uint32_t)q3, (uint32_t)(q3 >> 32)};
        __builtin_nontemporal_store(pa, r + 0);
        __builtin_nontemporal_store(pb, r + 1);
        __builtin_nontemporal_store(iv, r + 2);
    }
}

template <typename PairT>
__device__ inline uint32_t load_rec(const v4u32* r, PairT* q) {
    if constexpr (sizeof(PairT) == 4) {
        const v4u32 pv = __builtin_nontemporal_load(r + 0);
        q[0] = pv[0]; q[1] = pv[1]; q[2] = pv[2]; q[3] = pv[3];
        return __builtin_nontemporal_load(r + 1)[0];
    } else {
        const v4u32 pa = __builtin_nontemporal_load(r + 0), pb = __builtin_nontemporal_load(r + 1);
        q[0] = pa[0] | ((uint64_t)pa[1] << 32); q[1] = pa[2] | ((uint64_t)pa[3] << 32);
        q[2] = pb[0] | ((uint64_t)pb[1] << 32); q[3] = pb[2] | ((uint64_t)pb[3] << 32);
        return __builtin_nontemporal_load(r + 2)[0];
    }
}

}  // namespace lzg
