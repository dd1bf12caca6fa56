// enc.hip -- phase 2 of the encoder: the price-driven optimal parser and the
// range coder of src/main/java/SevenZip/Compression/LZMA/Encoder.java, one
// wavefront (kWave = 64 lanes) per independent stream.
//
// The parse is strictly serial per stream (adaptive probabilities and the
// price-table refresh schedule depend on every earlier symbol), so the GPU
// gets its throughput from many streams: a persistent grid pulls streams
// from a work queue (longest first). Inside a stream the wave's lanes run the
// data-parallel parts of getOptimum (Encoder.java:364-811):
//   * byte-compare loops (InWindow.GetMatchLen, InWindow.java:120-134):
//     kWave bytes per step + ballot,
//   * the per-length price loops for reps and matches (each length updates a
//     distinct _optimum slot, so lanes never collide; the ORDER between reps,
//     pairs and their look-ahead candidates is kept exactly as the reference
//     so strict-< ties resolve identically),
//   * literal prices (8 bit-prices summed across lanes),
//   * the periodic price-table refreshes (FillDistancesPrices,
//     FillAlignPrices, LenPriceTableEncoder.UpdateTable).
// Everything else is wave-uniform scalar code executed by all lanes in
// lockstep (so read-modify-writes of LDS state by all lanes are single
// updates). Register/LDS residency rules for this kernel:
//   * the per-stream state struct holds scalars and LDS pointers only (no
//     arrays), and every member is force-inlined, so it lives in registers;
//   * probability models, price tables, the match-info prefetch ring and
//     kOptLds _optimum entries (SoA) live in LDS: with fb <= 32 (RING) a
//     ring of the slots around the forward loop's position, whose evicted
//     entries go to a per-block HBM home; with fb > 32 the first kOptLds
//     slots, deeper ones in that HBM scratch behind an explicit fence;
//   * lanes exchange data through LDS only; a wavefront-scope fence orders
//     the compiler (LDS executes one wave's ops in order).
#include "lzma_common.h"
#include "runtime.h"

#include <type_traits>

// LZG_ENC_SLICED (enc_slice.hip): the same parser, compiled once more with the stop / resume
// of the sliced encode (lzma_enc_session_*) into namespace lzg::sliced. The product kernels
// of the batch encode keep their code and register allocation: the slicing is not in them.
#ifndef LZG_ENC_SLICED
#define LZG_ENC_SLICED 0
#endif

namespace lzg {
#if LZG_ENC_SLICED
namespace sliced {
#endif
constexpr bool kSliced = LZG_ENC_SLICED != 0;

static __constant__ Tables c_tab = make_tables();

constexpr int kOptLds = 64;         // _optimum slots kept in LDS (deeper slots spill to HBM); the LDS arrays
                                    // have one more slot, kOptLds, a sink for the writes of idle lanes
constexpr uint32_t kOptMask = kOptLds - 1;   // RING: slot i lives in entry i & kOptMask
constexpr uint32_t kFarEntry = kOptLds + 1;   // RING: the entry of slot cur + 65 until cur + 1 retires
static_assert((kOptLds & (kOptLds - 1)) == 0, "the _optimum ring is a power of two");
constexpr int kLitLdsMaxBits = 1;   // literal coders in LDS when lc + lp <= 1 (<= 3 KiB); else HBM/L2 ...
constexpr int kLitLdsMaxBitsFew = 3;   // ... or lc + lp <= 3 (12 KiB) when a launch has few streams per CU
constexpr int kFewStreams = 1024;      // "few": up to 4 streams per CU (LDS for 16 streams per CU is spoken for)
constexpr int kMdCap = kMatchMaxLen + 1;
constexpr int kRing = 32;           // match-info prefetch window (positions)
constexpr int kGW = 64;             // gather window: offsets -1 .. kGW-2 around the current position
constexpr int kGI = kGW / kWave;    // gather iterations per side (1 on hardware)
constexpr int kSides = 7;           // gathered sides: cur, rep0..rep3, pair0, pair1 (only cur's bytes go to LDS)
constexpr int kTpBytes = 2 * kNumFullDistances;   // tempPrices (u16 [kNumFullDistances]); the cur side's window aliases it
static_assert(kTpBytes >= kGW, "the gather window holds the cur side");
constexpr int kRbuf = 128;          // coder-record staging ring (records, power of two; halves of 64 go to HBM)
constexpr int kLitSlots = (8 + kWave - 1) / kWave;   // literal bits per lane (1 on hardware)
// _optimum's pp word: PosPrev (bits 0-11), PosPrev2 (12-23; slots < kNumOpts = 4096) and the
// flags Prev1IsChar | Prev2 << 1 (24-25). A candidate that clears Prev1IsChar writes the whole
// word (PosPrev2 and Prev2 are read only with Prev1IsChar set): no read-modify-write.
constexpr uint32_t kPosMask = 0xFFFu, kPos2Shift = 12, kFlagShift = 24;
static_assert(kNumOpts <= 4096, "PosPrev fits 12 bits");

#define FI __device__ __forceinline__
// Lanes of one wavefront exchange data through LDS. The hardware runs one
// wave's LDS instructions in order; this compiler barrier keeps the IR and
// machine schedulers from moving LDS accesses across an exchange point.
#define LANE_FENCE() asm volatile("" ::: "memory")
#define SPILL_FENCE() __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup")
// `for (v = lo + lane; v < hi; v += kWave)` with a wave-uniform trip count: the
// loop itself stays a scalar loop (a lane-dependent exit costs exec-mask
// bookkeeping on every iteration and makes values after it look per-lane).
#define LANE_FOR(T, v, lo, hi) \
    for (T v##_0 = (lo); v##_0 < (hi); v##_0 += kWave) if (const T v = v##_0 + (T)lane_id(); v < (hi))
// debug checkpoint (block 0, lane 0) into host-mapped memory
// (LZG_DEBUG builds only)
#ifdef LZG_DEBUG
#define DBG(k, v) do { if (dbg && blockIdx.x == 0 && lane_id() == 0) __hip_atomic_store(dbg + (k), (uint32_t)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)
#else
#define DBG(k, v) do {} while (0)
#endif
// Every loop is bounded: the forward loop by kNumOpts (cur < kNumOpts - 1 is checked), the
// coding loop by the stream length (every symbol advances now_pos by >= 1 or the stream ends).
// Phase profile (profiling build only, -DLZG_PROF): s_memtime cycles per phase,
// summed per stream into EncArgs::prof[stream * kProfSlots + phase].
#ifdef LZG_PROF
#define PCLK() __builtin_amdgcn_s_memtime()
#define PBEGIN(v) const uint64_t v = PCLK()
#define PEND(k, v) (prof[k] += PCLK() - (v))
#define PCOUNT(k) (prof[k]++)
#else
#define PBEGIN(v) do {} while (0)
#define PEND(k, v) do {} while (0)
#define PCOUNT(k) do {} while (0)
#endif

// A ballot over this wave's lanes. The CPU emulation (LZG_WAVE = 1) runs each wave as
// one lane: its own bit.
FI uint64_t wballot(bool p) {
#if LZG_WAVE == 1
    return p ? 1ull : 0ull;
#else
    return __ballot(p);
#endif
}

FI uint32_t uni32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }

FI uint64_t uni64(uint64_t v) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
}

// value of bit slot j (j < 8) held by lane j % kWave in register slot j / kWave
template <int N>
FI uint32_t lane_value(const uint32_t (&v)[N], int j) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v[j / kWave], j % kWave);
}

FI uint32_t brev32(uint32_t v) {
#if defined(__clang__)
    return __builtin_bitreverse32(v);
#else
    uint32_t r = 0;
    for (int i = 0; i < 32; i++) r |= ((v >> i) & 1u) << (31 - i);
    return r;
#endif
}

// GetPosSlot / GetPosSlot2 (Encoder.java:86-104) without the g_FastPos table:
// 2 floor(log2 pos) plus the bit below the leading one (pos >= 2)
FI uint32_t pos_slot(uint32_t pos) {
    if (pos < 2) return pos;
    const uint32_t n = 31u - (uint32_t)__clz((int)pos);
    return (n << 1) | ((pos >> (n - 1)) & 1u);
}

FI uint32_t sel4(uint32_t i, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return i == 0 ? a : (i == 1 ? b : (i == 2 ? c : d));
}

// FairPrio rows of the encoder's waves (lzma_common.h)
__device__ uint32_t g_enc_sched[kSchedRows * kSchedCols];

// The sliced encode's per-stream parser state in HBM (lzma_enc_session_*): everything of
// Encoder's that a CodeOneBlock boundary (Encoder.java:843-936, _additionalOffset == 0: no
// look-ahead pending, the _optimum path consumed) carries to the next block: the scalars
// (SS_* words), the probability models, the length-price tables with their countdowns and
// the distance / align price tables as last refreshed (the refresh schedule decides the
// output, so they are saved, not recomputed), and the literal coders. The decision-price
// cache (dmp) is a function of the models and is rebuilt.
enum { SL_SCALARS, SL_PROBS, SL_LENP, SL_LENC, SL_PSP, SL_DP, SL_AP, SL_LIT, SL_COUNT };
__host__ __device__ constexpr uint32_t slice_layout(uint32_t pb, uint32_t lc, uint32_t lp, uint32_t tsize, uint32_t* off) {
    const uint32_t sz[SL_COUNT] = {SS_WORDS * 4, prob_count(pb) * 2, 2 * (1u << pb) * tsize * 2, 2 * 16 * 4, 256 * 2,
                                   512 * 2, 16 * 4, (0x300u << (lc + lp)) * 2};
    uint32_t o = 0;
    for (int i = 0; i < SL_COUNT; i++) { if (off) off[i] = o; o += (sz[i] + 15) & ~15u; }
    return o;
}

template <typename PairT, bool LIT_LDS, int PBS, bool RING>
struct Enc {
    using PP = PairPack<PairT>;
    using PL = ProbLayout<PBS>;
    static constexpr int E_IS_MATCH = PL::IS_MATCH, E_IS_REP = PL::IS_REP, E_G0 = PL::G0, E_G1 = PL::G1,
                         E_G2 = PL::G2, E_R0L = PL::R0L, E_PSLOT = PL::PSLOT, E_PENC = PL::PENC,
                         E_ALIGN = PL::ALIGN, E_LEN = PL::LEN, E_RLEN = PL::RLEN, E_LOW = PL::LOW,
                         E_MID = PL::MID, E_HIGH = PL::HIGH, E_COUNT = PL::COUNT;
    uint32_t lane_v;          // threadIdx.x: read through lane_id()
    // The lane index. In the kernels whose literal coders live in HBM (many streams per CU:
    // 16 per CU, a 128-VGPR budget) it is made opaque to the optimizer once per coded symbol
    // and once per forward position (refresh_lane): otherwise LICM hoists every lane-derived
    // value (lane + c, lane == c, 7 - (lane & 7), ...) of the whole kernel to its entry, where
    // hundreds of them hold VGPRs and SGPR pairs for the kernel's lifetime and spilled to
    // scratch (128 VGPRs + scratch -> 56 VGPRs, none; 4096 streams 569 -> 537 ms). Opaque at
    // every use instead, each use recomputed its value (432 instructions per byte); once per
    // iteration, the values are shared within the iteration: 60 VGPRs, 4096 streams
    // 532 -> 522 ms (profiles/r05/ab_parse_lane_refresh.jsonl). With the literal coders in LDS
    // (few streams per CU, the budget the LDS leaves is larger) the hoisted values fit, and
    // recomputing them cost one stream 5 %.
    FI uint32_t lane_id() const { return lane_v; }
    FI void refresh_lane() {
#if LZG_WAVE == 64
        if constexpr (!LIT_LDS) asm volatile("" : "+v"(lane_v));
#endif
    }
    // ---- LDS
    uint16_t* pp;             // ProbPrices [512]
    uint16_t* probs;          // fixed models (lzma_common.h layout)
    uint32_t* dmp;            // price cache of the decision models (isMatch .. isRep0Long, indices < E_PSLOT):
                              // price0 | price1 << 16, rewritten by the coder whenever it adapts one
    uint16_t* lit;            // literal coders (LDS or HBM by LIT_LDS)
    uint16_t* lenp;           // [2][npos * tsize]
    uint32_t* lenc;           // [2][16]
    uint16_t* psp;            // _posSlotPrices [256] (prices < 2^14: 16 bits suffice)
    uint16_t* dp;             // _distancesPrices [512]
    uint32_t* ap;             // _alignPrices [16]
    uint16_t* tp;             // tempPrices [128]
    const PairT* mdp;         // the current position's pairs (packed): its ring slot, or md_buf
    PairT* md_buf;            // a copy when the list is longer than the inline pairs or is clamped
    uint8_t* win;             // gather window: the cur side's bytes at offsets -1 .. kGW - 2 (aliased by tp)
    uint32_t* ring_info;      // [kRing]
    PairT* ring_pairs;        // [kRing * kInlinePairs]
    uint32_t* o_price;        // _optimum SoA, [kOptLds] each (+ the sink entry, + kFarEntry)
    uint32_t* o_pp;
    int32_t* o_bp;
    int32_t* o_bp2;
    uint32_t* o_backs;        // [kOptLds][4] (one 16-byte record per slot: Backs0..3)
    uint32_t* o_bytes;        // [kOptLds] cur byte | match byte << 8 | previous byte << 16 of each parsed
                              // position, so the coder needs no HBM byte loads (RING: | state << 24)
    uint16_t* rbuf;           // coder-record staging ring [kRbuf]
    __amdgpu_buffer_rsrc_t spill;   // _optimum slots >= kOptLds in HBM (9 fields x kNumOpts dwords)
    // ---- parameters
    uint32_t fb, lc, lp, pb, ps_mask, eos, dist_table_size, tsize;
    // ---- stream
    const uint8_t* in;
    __amdgpu_buffer_rsrc_t inb;   // the stream's bytes, range-checked (out of range reads 0, never fault)
    uint32_t n;
    uint32_t bad;                 // internal-consistency watchdog tripped (reason code, 0 = fine)
    uint32_t* dbg;
    uint16_t* recs;           // the stream's coder records in HBM (rc.hip codes them)
    uint64_t rcap, rpos;      // record capacity / records emitted
    uint32_t overflow;
    const v4u32* pairs;        // per-position match-list records
    const uint32_t* ovf_off;
    const PairT* ovf;
    uint64_t gbase;
    uint32_t ring_base;
    // ---- Encoder fields (Encoder.java:132-181)
    uint32_t mfpos;           // match-finder position, 0-based (BinTree._pos - 1)
    int32_t additional_offset, opt_end, opt_cur;
    uint32_t longest_found, longest_len, num_pairs;
    uint32_t state, prev_byte;
    uint32_t rd0, rd1, rd2, rd3;   // _repDistances
    uint32_t rp0, rp1, rp2, rp3;   // reps
    uint32_t match_price_count, align_price_count;
    // ---- RING bookkeeping of _optimum (see the accessors)
    uint32_t ring_top;        // highest slot whose ahead fields are in the ring
    uint32_t far_valid;       // slot cur + 65 is held in the far entry (kFarEntry)
    // State that no loop reads, kept in LDS instead of registers (the kernel is at its SGPR
    // limit): FairPrio's (read once per 1/256 of the stream)
    struct Cold {
        FairPrio prio;
    };
    Cold* cold;
    // ---- the sliced encode (kSliced kernels only): the stream's state region, where to stop
    uint8_t* sst;
    uint32_t sstop, sresume;
    // ---- per-position gather (see gather()): p = current position, equality masks per side
    uint32_t gp;
    // RING (fb <= 32): 32-bit masks, bit k = offset k (0 .. 31), enough for every length up
    // to fb; one scalar register each instead of two (the kernel is at its SGPR limit).
    // Otherwise 64-bit masks, bit k = offset k - 1 (-1 .. 62). Compares past the window
    // continue with match_len either way.
    using GM = typename std::conditional<RING, uint32_t, uint64_t>::type;
    static constexpr int kMB = RING ? 32 : 64;   // mask bits
    static constexpr int kMO = RING ? 0 : 1;     // the bit of offset 0
    GM gm0, gm1, gm2, gm3, gmp0, gmp1;
    uint32_t g_prev, g_cur, g_mb;   // bytes at p - 1 and p, and at p - rep0 - 1 (the match byte), from the gather
#ifdef LZG_PROF
    uint64_t prof[kProfSlots];
#endif

    // ------------------------------------------------------------ _optimum
    // The spill side goes through a buffer descriptor (buffer_load/store), an
    // access kind the compiler cannot merge with the LDS side into one generic
    // (flat) pointer. Byte offsets inside the per-block spill region:
    //   price | pp | bp | bp2 | fs | backs[4] | bytes, kNumOpts dwords each.
    FI uint32_t sload(uint32_t field, uint32_t i) const {
        return __builtin_amdgcn_raw_buffer_load_b32(spill, (field * kNumOpts + i) * 4, 0, 0);
    }
    FI void sstore(uint32_t field, uint32_t i, uint32_t v) {
        __builtin_amdgcn_raw_buffer_store_b32(v, spill, (field * kNumOpts + i) * 4, 0, 0);
    }
    // Which copy of slot i is current. Non-RING (fb > 32): slots < kOptLds in
    // LDS, deeper ones in HBM. RING (fb <= 32): one forward step reads slots
    // >= cur - 65 and writes slots <= cur + 65 (lenTest, lenTest2 <= fb), so
    // LDS holds a ring: the "ahead" fields (price, pp, bp, bp2, flags) of the
    // slots (ring_top - 64, ring_top] and the "behind" fields (backs, bytes |
    // state << 24) of (top - 64, top], top the last slot a step wrote. An
    // entry is written back to the slot's HBM home (field layout as the spill
    // scratch) before the ring reuses it; Backward, the cached path and the
    // coder read older slots there. F: the caller knows the slot is in LDS.
    FI bool a_in(uint32_t i) const { return RING ? i + (uint32_t)kOptLds > ring_top : i < (uint32_t)kOptLds; }
    // top: the highest slot whose behind fields were written (cur - 1 in a forward
    // step, opt_end - 1 once the parse has ended)
    FI bool b_in(uint32_t i, uint32_t top) const { return RING ? i + (uint32_t)kOptLds > top : i < (uint32_t)kOptLds; }
    static FI uint32_t ix(uint32_t i) { return RING ? (i & kOptMask) : i; }
    template <bool F = false> FI uint32_t price_at(uint32_t i) const { if (F || a_in(i)) return o_price[ix(i)]; return sload(0, i); }
    template <bool F = false> FI void set_price(uint32_t i, uint32_t v) { if (F || a_in(i)) o_price[ix(i)] = v; else sstore(0, i, v); }
    template <bool F = false> FI uint32_t pp_at(uint32_t i) const { if (F || a_in(i)) return o_pp[ix(i)]; return sload(1, i); }
    template <bool F = false> FI void set_pp(uint32_t i, uint32_t v) { if (F || a_in(i)) o_pp[ix(i)] = v; else sstore(1, i, v); }
    template <bool F = false> FI int32_t bp_at(uint32_t i) const { if (F || a_in(i)) return o_bp[ix(i)]; return (int32_t)sload(2, i); }
    template <bool F = false> FI void set_bp(uint32_t i, int32_t v) { if (F || a_in(i)) o_bp[ix(i)] = v; else sstore(2, i, (uint32_t)v); }
    template <bool F = false> FI int32_t bp2_at(uint32_t i) const { if (F || a_in(i)) return o_bp2[ix(i)]; return (int32_t)sload(3, i); }
    template <bool F = false> FI void set_bp2(uint32_t i, int32_t v) { if (F || a_in(i)) o_bp2[ix(i)] = v; else sstore(3, i, (uint32_t)v); }
    // the flags (Prev1IsChar = bit 0, Prev2 = bit 1, Optimal.java:8-9) ride in pp's top byte
    template <bool F = false> FI uint32_t fs_at(uint32_t i) const { return pp_at<F>(i) >> kFlagShift; }
    // behind fields: in RING mode a home read waits for the write-backs (rare: a
    // path back by 65 slots, or a coded literal 64 slots behind the parse end)
    template <bool F = false> FI uint32_t back_at(uint32_t i, int k, uint32_t top) const {
        if (F || b_in(i, top)) return o_backs[ix(i) * 4 + k];
        if (RING) SPILL_FENCE();
        return sload(5 + k, i);
    }
    template <bool F = false> FI void set_back(uint32_t i, int k, uint32_t v) {
        if (F || RING || i < (uint32_t)kOptLds) o_backs[ix(i) * 4 + k] = v; else sstore(5 + k, i, v);
    }
    // all four Backs of slot i: one 16-byte LDS access (or the HBM home, as back_at)
    template <bool F = false> FI v4u32 backs4_at(uint32_t i, uint32_t top) const {
        if (F || b_in(i, top)) return *(const v4u32*)(o_backs + ix(i) * 4);
        if (RING) SPILL_FENCE();
        const v4u32 v = {sload(5, i), sload(6, i), sload(7, i), sload(8, i)};
        return v;
    }
    template <bool F = false> FI void set_backs4(uint32_t i, uint32_t b0, uint32_t b1, uint32_t b2, uint32_t b3) {
        if (F || RING || i < (uint32_t)kOptLds) {
            const v4u32 v = {b0, b1, b2, b3};
            *(v4u32*)(o_backs + ix(i) * 4) = v;
        } else { sstore(5, i, b0); sstore(6, i, b1); sstore(7, i, b2); sstore(8, i, b3); }
    }
    template <bool F = false> FI uint32_t bytes_at(uint32_t i, uint32_t top) const {
        if (F || b_in(i, top)) return o_bytes[ix(i)];
        if (RING) SPILL_FENCE();
        return sload(9, i);
    }
    template <bool F = false> FI void set_bytes(uint32_t i, uint32_t v) {
        if (F || RING || i < (uint32_t)kOptLds) o_bytes[ix(i)] = v; else sstore(9, i, v);
    }
    // the State of slot i's best path
    template <bool F = false> FI uint32_t state_at(uint32_t i, uint32_t top) const { return bytes_at<F>(i, top) >> 24; }
    // RING: write back the ahead fields of slot i (its entry is about to hold i + 64)
    FI void evict_ahead(uint32_t i) {
        const uint32_t r = i & kOptMask;
        LANE_FOR(uint32_t, k, 0u, 3u) {
            const uint32_t v = k == 0 ? o_pp[r] : (k == 1 ? (uint32_t)o_bp[r] : (uint32_t)o_bp2[r]);
            sstore(1 + k, i, v);
        }
    }
    // RING: write back the behind fields of slot i
    FI void evict_behind(uint32_t i) {
        const uint32_t r = i & kOptMask;
        LANE_FOR(uint32_t, k, 0u, 5u) sstore(5 + k, i, k < 4 ? o_backs[r * 4 + k] : o_bytes[r]);
    }
    // pair k of the current position's match list
    FI uint32_t md_l(uint32_t k) const { return PP::len(mdp[k]); }
    FI uint32_t md_d(uint32_t k) const { return PP::dist(mdp[k]); }
    FI uint32_t win_bytes() const { return g_cur | (g_mb << 8) | (g_prev << 16); }
    template <bool F = false> FI uint32_t pos_prev(uint32_t i) const { return pp_at<F>(i) & kPosMask; }
    template <bool F = false> FI uint32_t pos_prev2(uint32_t i) const { return (pp_at<F>(i) >> kPos2Shift) & kPosMask; }
    // after lanes wrote slots up to `hi`, make them visible to every lane
    FI void fence_upto(uint32_t hi) {
        LANE_FENCE();
#ifndef LZG_ABL_NOFENCE
        if (!RING && hi >= (uint32_t)kOptLds) SPILL_FENCE();
#endif
    }

    // ------------------------------------------------------------ prices
    FI uint32_t price_bit(uint32_t prob, uint32_t bit) const { return pp[(((prob - bit) ^ (0u - bit)) & 2047u) >> 2]; }
    FI uint32_t price0(uint32_t prob) const { return pp[prob >> 2]; }
    FI uint32_t price1(uint32_t prob) const { return pp[(kBitModelTotal - prob) >> 2]; }
    // one LDS read per decision price (no prob -> ProbPrices chain)
    FI uint32_t dm0(uint32_t i) const { return dmp[i] & 0xFFFFu; }
    FI uint32_t dm1(uint32_t i) const { return dmp[i] >> 16; }
    FI uint32_t dmb(uint32_t i, uint32_t bit) const { return bit ? dm1(i) : dm0(i); }
    FI uint32_t bt_price(const uint16_t* p, int nbits, uint32_t sym) const {   // BitTreeEncoder.java:38-48
        uint32_t price = 0, m = 1;
        for (int b = nbits; b != 0;) { b--; uint32_t bit = (sym >> b) & 1; price += price_bit(p[m], bit); m = (m << 1) + bit; }
        return price;
    }
    FI uint32_t rev_price(const uint16_t* p, int nbits, uint32_t sym) const {  // BitTreeEncoder.java:50-60
        uint32_t price = 0, m = 1;
        for (int i = nbits; i != 0; i--) { uint32_t bit = sym & 1; sym >>= 1; price += price_bit(p[m], bit); m = (m << 1) | bit; }
        return price;
    }
    FI uint16_t* lit_coder(uint32_t pos, uint32_t prev) const {   // LiteralEncoder.GetSubCoder (:93-95)
        uint32_t idx = ((pos & ((1u << lp) - 1)) << lc) + (prev >> (8 - lc));
        return lit + (size_t)idx * 0x300;
    }
    // LiteralEncoder.Encoder2.GetPrice (LiteralEncoder.java:42-64): one bit per lane.
    FI uint32_t lit_price(const uint16_t* p, bool match_mode, uint32_t mb, uint32_t sym) const {
        uint32_t price = 0;
        int first = -1;
        if (match_mode) {
            uint32_t diff = (mb ^ sym) & 0xFFu;
            first = diff ? 31 - __clz(diff) : -1;
        }
#if LZG_WAVE == 64
        {   // every lane computes bit (lane & 7): no exec-mask bookkeeping on the scalar unit;
            // lanes 8-63 repeat lanes 0-7's addresses and their prices are dropped
            const int i = 7 - (int)(lane_id() & 7u);
            const uint32_t bit = (sym >> i) & 1;
            const uint32_t ctx = (0x100u | sym) >> (i + 1);
            const uint32_t idx = (match_mode && i >= first) ? ((1 + ((mb >> i) & 1)) << 8) + ctx : ctx;
            const uint32_t pr = price_bit(p[idx], bit);
            price = lane_id() < 8 ? pr : 0u;
        }
#else
        LANE_FOR(int, j, 0, 8) {
            int i = 7 - j;
            uint32_t bit = (sym >> i) & 1;
            uint32_t ctx = (0x100u | sym) >> (i + 1);
            uint32_t idx = ctx;
            if (match_mode && i >= first) idx = ((1 + ((mb >> i) & 1)) << 8) + ctx;
            price += price_bit(p[idx], bit);
        }
#endif
#if LZG_WAVE == 64
        // sum of lanes 0-7 without LDS traffic: DPP quad swaps, then a rotate by 4
        // within the 16-lane row; lane 0 holds the total (readlane keeps it scalar)
        price += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)price, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
        price += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)price, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
        price += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)price, 0x12C, 0xF, 0xF, false);  // row_ror:12 (lane i reads lane i+4)
        return (uint32_t)__builtin_amdgcn_readlane((int)price, 0);
#else
        for (int o = 1; o < 8 && o < kWave; o <<= 1) price += __shfl_xor(price, o);
        return (uint32_t)__builtin_amdgcn_readfirstlane((int)price);
#endif
    }
    FI uint32_t len_price(int which, uint32_t sym, uint32_t ps) const {
        return lenp[(which << pb) * tsize + ps * tsize + sym];
    }

    // ------------------------------------------------------------ window (InWindow.java:115-138)
    FI uint32_t in_byte(uint32_t off) const { return __builtin_amdgcn_raw_buffer_load_b8(inb, off, 0, 0); }
    FI uint32_t byte_at(int32_t index) const { return in_byte(mfpos + (uint32_t)index); }
    FI uint32_t avail() const { return n - mfpos; }
    FI uint32_t match_len(int32_t index, uint32_t distance, int32_t limit) {
        int64_t p0 = (int64_t)mfpos + index;
        if (p0 + limit > (int64_t)n) limit = (int32_t)((int64_t)n - p0);
        if (limit <= 0) return 0;
        const uint32_t a = (uint32_t)p0, b = (uint32_t)p0 - (distance + 1);
        for (int32_t i0 = 0; i0 < limit; i0 += kWave) {
            int32_t i = i0 + (int32_t)lane_id();
            bool ne = i < limit ? (in_byte(a + (uint32_t)i) != in_byte(b + (uint32_t)i)) : true;
            uint64_t m = wballot(ne);
            if (m) {
                int32_t r = i0 + (__ffsll((long long)m) - 1);
                return (uint32_t)(r < limit ? r : limit);
            }
        }
        return (uint32_t)limit;
    }

    // ------------------------------------------------------------ per-position gather
    // Every byte compare of one parse position (InWindow.GetMatchLen calls at
    // Encoder.java:393-399, 631-700, 759-772) reads the window at offsets
    // o = -1 .. kGW-2 from p (the current byte) on the cur side and at
    // p + o - dist - 1 on the rep / match sides. gather() issues all of those
    // byte loads at once (one lane per offset, one memory round trip), keeps
    // equality masks per side (bit o+1 = bytes equal at offset o), keeps the three
    // bytes the position step prices its literal with in scalars and the cur side's
    // bytes in LDS (two-step literals). Compares past the window fall back to match_len.
    FI void gather(bool with_pairs) {
        gp = mfpos - 1;
        const uint32_t d0 = rp0 + 1, d1 = rp1 + 1, d2 = rp2 + 1, d3 = rp3 + 1;
        const uint32_t e0 = num_pairs > 0 ? md_d(0) + 1 : d0, e1 = num_pairs > 1 ? md_d(1) + 1 : d0;
        uint32_t va[kGI], v0[kGI], v1[kGI], v2[kGI], v3[kGI], w0[kGI], w1[kGI];
#pragma unroll
        for (int it = 0; it < kGI; it++) {
            const uint32_t q = gp - 1 + (uint32_t)(it * kWave) + lane_id();
            va[it] = in_byte(q);
            v0[it] = in_byte(q - d0); v1[it] = in_byte(q - d1); v2[it] = in_byte(q - d2); v3[it] = in_byte(q - d3);
            if (with_pairs) { w0[it] = in_byte(q - e0); w1[it] = in_byte(q - e1); }
        }
        uint64_t m0 = 0, m1 = 0, m2 = 0, m3 = 0, mp0 = 0, mp1 = 0;   // bit k: offset k - 1
#pragma unroll
        for (int it = 0; it < kGI; it++) {
            const int sh = it * kWave;
            const uint32_t k = (uint32_t)sh + lane_id();
            m0 |= (uint64_t)wballot(va[it] == v0[it]) << sh;
            m1 |= (uint64_t)wballot(va[it] == v1[it]) << sh;
            m2 |= (uint64_t)wballot(va[it] == v2[it]) << sh;
            m3 |= (uint64_t)wballot(va[it] == v3[it]) << sh;
            if (with_pairs) {
                mp0 |= (uint64_t)wballot(va[it] == w0[it]) << sh;
                mp1 |= (uint64_t)wballot(va[it] == w1[it]) << sh;
            }
            win[k] = (uint8_t)va[it];   // the cur side only: the other sides' bytes are read (rarely, by a
                                         // two-step candidate's literal) straight from the stream
        }
        constexpr int drop = 1 - kMO;   // RING: offset -1's bit goes
        gm0 = (GM)(m0 >> drop); gm1 = (GM)(m1 >> drop); gm2 = (GM)(m2 >> drop); gm3 = (GM)(m3 >> drop);
        gmp0 = (GM)(mp0 >> drop); gmp1 = (GM)(mp1 >> drop);
        // the three bytes every position step reads, straight from the loaded registers
        // (offsets -1 and 0 are window entries 0 and 1): no LDS round trip on the chain
        g_prev = lane_value(va, 0);
        g_cur = lane_value(va, 1);
        g_mb = lane_value(v0, 1);
        LANE_FENCE();
    }
    // byte at p + o on the cur side
    // byte at p + o on the cur side (a two-step candidate's literal)
    FI uint32_t a_byte(int32_t o) const {
        return (o >= -1 && o <= kGW - 2) ? (uint32_t)win[o + 1] : in_byte(gp + (uint32_t)o);
    }
    // byte at p + o - dist - 1 (side 1..6 = rep0..3, pair0..1; side < 0: not gathered); only a
    // two-step candidate's literal reads one (a few percent of the positions): from the stream
    FI uint32_t b_byte(int side, uint32_t dist, int32_t o) const {
        (void)side;
        return in_byte(gp + (uint32_t)o - dist - 1);
    }
    // InWindow.GetMatchLen(index = o - 1, dist, limit) from the side's mask; the
    // part of the compare beyond the window continues with match_len.
    FI uint32_t glen(GM m, uint32_t dist, int32_t o, int32_t limit) {
        const int64_t rem = (int64_t)n - ((int64_t)gp + o);
        if (limit > rem) limit = (int32_t)rem;
        if (limit <= 0) return 0;
        const int b = o + kMO;                     // 0 <= b
        uint32_t r;
        if (b >= kMB) r = 0;
        else {
            const GM x = (GM)~m >> b;              // bits past the window shift in as 0 (= "equal")
            const uint32_t lim_w = (uint32_t)(kMB - b);
            r = x ? (uint32_t)(RING ? __builtin_ctz((uint32_t)x) : __builtin_ctzll((uint64_t)x)) : (uint32_t)kMB;
            if (r > lim_w) r = lim_w;
        }
        if (r >= (uint32_t)limit) return (uint32_t)limit;
        if ((uint32_t)b + r < (uint32_t)kMB) return r;   // mismatch inside the window
        return r + match_len(o + (int32_t)r - 1, dist, limit - (int32_t)r);
    }
    // the mask bits of offsets o and o + 1 both set (true past the window: no pre-check there)
    static FI bool eq2(GM m, uint32_t o) { return o + 1 + kMO >= (uint32_t)kMB || ((m >> (o + kMO)) & 3u) == 3u; }
    static FI bool eq1(GM m, uint32_t o) { return ((m >> (o + kMO)) & 1u) != 0; }   // o + kMO < kMB

    // ------------------------------------------------------------ coder records
    // The range coder (RangeEncoder.java:38-87) does not feed back into the
    // parse: its arithmetic needs only each decision's probability before the
    // update and the bit. The parser therefore emits one 16-bit record per
    // binary decision (prob | bit << 11; prob 0 = a direct bit) and rc.hip runs
    // the coder arithmetic, one lane per stream, on the vector unit. Records
    // are staged in LDS and written 64 at a time by 32 lanes (one 128-byte
    // store): a global store per symbol would make the next dependent load
    // wait for it (vmcnt counts stores and loads alike on CDNA).
    FI void rec_store_block(uint64_t blk) {   // records [blk * 64, blk * 64 + 64): a full half of the ring
        if ((blk + 1) * 64 > rcap) { overflow = 1; return; }
        const uint32_t* src = (const uint32_t*)(rbuf + (blk & 1) * 64);
        uint32_t* dst = (uint32_t*)(recs + blk * 64);
        LANE_FOR(uint32_t, w, 0u, 32u) __builtin_nontemporal_store(src[w], dst + w);
    }
    FI void rec_store_tail() {   // the partial block at the end of the stream
        const uint64_t blk = rpos >> 6;
        const uint32_t cnt = (uint32_t)rpos & 63u;
        if (cnt == 0) return;
        if (blk * 64 + cnt > rcap) { overflow = 1; return; }
        LANE_FOR(uint32_t, k, 0u, cnt) __builtin_nontemporal_store(rbuf[(blk & 1) * 64 + k], recs + blk * 64 + k);
        LANE_FENCE();
    }
    // ------------------------------------------------------------ symbol coder
    // One coded symbol (literal, rep, match or the end marker) is the sequence
    // of binary decisions Encoder.java:890-1024 / :818-835 make. Within one
    // symbol every decision uses a distinct probability (bit-tree nodes along
    // one path are distinct, each model is visited at most once), so the
    // decisions are laid out one per lane (q_* below), every lane loads its
    // probability at once, the range coder (RangeEncoder.Encode/
    // EncodeDirectBits, RangeEncoder.java:38-77) runs serially over the
    // register copies, and the lanes write the adapted probabilities back at
    // once. The coder loop is the only range-coder instance in the kernel.
    static constexpr int kQS = (64 + kWave - 1) / kWave;   // decision slots per lane (1 on hardware)
    enum : uint32_t { QK_NONE = 0, QK_PROB = 1, QK_LIT = 2, QK_DIRECT = 3 };
    struct Q {
        uint32_t n;
        uint32_t idx[kQS], bit[kQS], kind[kQS];
    };
    FI void q_init(Q& q) const {
        q.n = 0;
#pragma unroll
        for (int t = 0; t < kQS; t++) { q.idx[t] = 0; q.bit[t] = 0; q.kind[t] = QK_NONE; }
    }
    // one decision against probs[index]
    FI void q_bit(Q& q, uint32_t index, uint32_t bit) const {
#pragma unroll
        for (int t = 0; t < kQS; t++) {   // selects, not a branch: the exec-mask juggling runs on the scalar unit
            const bool m = (uint32_t)(t * kWave) + lane_id() == q.n;
            q.idx[t] = m ? index : q.idx[t];
            q.bit[t] = m ? bit : q.bit[t];
            q.kind[t] = m ? (uint32_t)QK_PROB : q.kind[t];
        }
        q.n++;
    }
    // BitTreeEncoder.Encode (BitTreeEncoder.java:18-27): node of bit i (MSB first) = the i-bit prefix
    FI void q_bt(Q& q, uint32_t base, uint32_t nbits, uint32_t sym) const {
#pragma unroll
        for (int t = 0; t < kQS; t++) {
            const uint32_t i = (uint32_t)(t * kWave) + lane_id() - q.n;
            const bool m = i < nbits;
            const uint32_t ic = m ? i : 0u;
            q.idx[t] = m ? base + ((sym | (1u << nbits)) >> (nbits - ic)) : q.idx[t];
            q.bit[t] = m ? (sym >> (nbits - 1 - ic)) & 1u : q.bit[t];
            q.kind[t] = m ? (uint32_t)QK_PROB : q.kind[t];
        }
        q.n += nbits;
    }
    // BitTreeEncoder.ReverseEncode (BitTreeEncoder.java:29-36, Encoder.java:196-205): bit i (LSB first)
    // at node 1 followed by bits 0..i-1
    FI void q_rev(Q& q, uint32_t base, uint32_t nbits, uint32_t sym) const {
#pragma unroll
        for (int t = 0; t < kQS; t++) {
            const uint32_t i = (uint32_t)(t * kWave) + lane_id() - q.n;
            const bool in = i < nbits;
            const uint32_t ic = in ? i : 0u;
            const uint32_t m = (1u << ic) | (ic ? brev32(sym) >> (32 - ic) : 0u);
            q.idx[t] = in ? base + m : q.idx[t];
            q.bit[t] = in ? (sym >> ic) & 1u : q.bit[t];
            q.kind[t] = in ? (uint32_t)QK_PROB : q.kind[t];
        }
        q.n += nbits;
    }
    // RangeEncoder.EncodeDirectBits (RangeEncoder.java:41-51), MSB first
    FI void q_direct(Q& q, uint32_t v, uint32_t nbits) const {
#pragma unroll
        for (int t = 0; t < kQS; t++) {
            const uint32_t i = (uint32_t)(t * kWave) + lane_id() - q.n;
            const bool m = i < nbits;
            q.bit[t] = m ? (v >> (nbits - 1 - (m ? i : 0u))) & 1u : q.bit[t];
            q.kind[t] = m ? (uint32_t)QK_DIRECT : q.kind[t];
        }
        q.n += nbits;
    }
    // LiteralEncoder.Encoder2.Encode / EncodeMatched (LiteralEncoder.java:17-40) against the
    // coder at lit[base]: matched context while every higher bit equals the match byte's
    FI void q_lit(Q& q, uint32_t base, bool matched, uint32_t mb, uint32_t sym) const {
        int first = -1;
        if (matched) {
            const uint32_t diff = (mb ^ sym) & 0xFFu;
            first = diff ? 31 - __clz(diff) : -1;
        }
#pragma unroll
        for (int t = 0; t < kQS; t++) {
            const uint32_t j = (uint32_t)(t * kWave) + lane_id() - q.n;
            const bool m = j < 8u;
            const int i = 7 - (int)(j & 7u);
            const uint32_t ctx = (0x100u | sym) >> (i + 1);
            q.idx[t] = m ? base + ((matched && i >= first) ? ((1 + ((mb >> i) & 1)) << 8) + ctx : ctx) : q.idx[t];
            q.bit[t] = m ? (sym >> i) & 1u : q.bit[t];
            q.kind[t] = m ? (uint32_t)QK_LIT : q.kind[t];
        }
        q.n += 8;
    }
    // LenEncoder.Encode (LenEncoder.java:24-39)
    FI void q_len(Q& q, int which, uint32_t sym, uint32_t ps) const {
        const uint32_t L = which ? E_RLEN : E_LEN;
        if (sym < (uint32_t)kNumLowLenSymbols) { q_bit(q, L + LEN_CHOICE, 0); q_bt(q, L + E_LOW + ps * 8, 3, sym); }
        else {
            sym -= kNumLowLenSymbols;
            q_bit(q, L + LEN_CHOICE, 1);
            if (sym < (uint32_t)kNumMidLenSymbols) { q_bit(q, L + LEN_CHOICE + 1, 0); q_bt(q, L + E_MID + ps * 8, 3, sym); }
            else { q_bit(q, L + LEN_CHOICE + 1, 1); q_bt(q, L + E_HIGH, 8, sym - kNumMidLenSymbols); }
        }
    }
    // has_lit (wave-uniform): the symbol codes a literal. Only then do the lanes load and
    // store the literal coders (HBM): a global store of the other symbols would make the
    // next load on the chain wait for it (vmcnt counts stores and loads alike).
    FI void q_run(const Q& q, bool has_lit) {
        // branch-free: every lane loads and stores; lanes whose slot is not of a kind use the
        // sink entry past that table (lit: nlit, probs: E_COUNT, dmp: E_PSLOT, rbuf: kRbuf)
        const uint32_t nlit = 0x300u << (lc + lp);
        uint32_t pr[kQS];
#pragma unroll
        for (int t = 0; t < kQS; t++) {
            const bool isl = q.kind[t] == QK_LIT, isp = q.kind[t] == QK_PROB;
            const uint32_t lv = has_lit ? (uint32_t)lit[isl ? q.idx[t] : nlit] : 0u;
            const uint32_t pv = probs[isp ? q.idx[t] : (uint32_t)E_COUNT];
            pr[t] = isl ? lv : (isp ? pv : 0u);
        }
        const uint32_t base = (uint32_t)rpos;
#pragma unroll
        for (int t = 0; t < kQS; t++) {
            const uint32_t j = (uint32_t)(t * kWave) + lane_id();
            const bool isl = q.kind[t] == QK_LIT, isp = q.kind[t] == QK_PROB;
            rbuf[j < q.n ? (base + j) & (kRbuf - 1) : (uint32_t)kRbuf] =
                (uint16_t)((q.kind[t] == QK_DIRECT ? 0u : pr[t]) | (q.bit[t] << 11));
            const uint32_t p = pr[t];
            const uint16_t np = (uint16_t)(q.bit[t] ? p - (p >> kNumMoveBits) : p + ((kBitModelTotal - p) >> kNumMoveBits));
#ifdef LZG_ABL_LITSTORE
            if (has_lit) lit[nlit] = np;   // ablation: literal models never adapt
#else
            if (has_lit) lit[isl ? q.idx[t] : nlit] = np;
#endif
            probs[isp ? q.idx[t] : (uint32_t)E_COUNT] = np;
            dmp[(isp && q.idx[t] < (uint32_t)E_PSLOT) ? q.idx[t] : (uint32_t)E_PSLOT] = price0(np) | (price1(np) << 16);
        }
        LANE_FENCE();
        const uint64_t p0 = rpos;
        rpos += q.n;   // q.n <= 48 < 64: at most one block completes per symbol
        if ((p0 >> 6) != (rpos >> 6)) rec_store_block(p0 >> 6);
    }

    // ------------------------------------------------------------ price tables
    FI void update_len_table(int which, uint32_t ps) {   // LenEncoder.SetPrices + LenPriceTableEncoder.UpdateTable
        const uint16_t* L = probs + (which ? E_RLEN : E_LEN);
        uint32_t a0 = price0(L[LEN_CHOICE]), a1 = price1(L[LEN_CHOICE]);
        uint32_t b0 = a1 + price0(L[LEN_CHOICE + 1]), b1 = a1 + price1(L[LEN_CHOICE + 1]);
        uint16_t* dst = lenp + (which << pb) * tsize + ps * tsize;
        LANE_FOR(uint32_t, i, 0u, tsize) {
            uint32_t pr;
            if (i < (uint32_t)kNumLowLenSymbols) pr = a0 + bt_price(L + E_LOW + ps * 8, 3, i);
            else if (i < (uint32_t)(kNumLowLenSymbols + kNumMidLenSymbols)) pr = b0 + bt_price(L + E_MID + ps * 8, 3, i - kNumLowLenSymbols);
            else pr = b1 + bt_price(L + E_HIGH, 8, i - kNumLowLenSymbols - kNumMidLenSymbols);
            dst[i] = (uint16_t)pr;
        }
        lenc[which * 16 + ps] = tsize;
        LANE_FENCE();
    }
    FI void fill_distances_prices() {   // Encoder.java:1087-1118
        LANE_FOR(uint32_t, i, (uint32_t)kStartPosModelIndex, (uint32_t)kNumFullDistances) {
            uint32_t ps = pos_slot(i), footer = (ps >> 1) - 1, base = (2 | (ps & 1)) << footer;
            tp[i] = (uint16_t)rev_price(probs + E_PENC + (int32_t)(base - ps - 1), (int)footer, i - base);
        }
        for (uint32_t l = 0; l < (uint32_t)kNumLenToPosStates; l++) {
            uint32_t st = l << kNumPosSlotBits;
            LANE_FOR(uint32_t, ps, 0u, dist_table_size) {
                uint32_t pr = bt_price(probs + E_PSLOT + st, kNumPosSlotBits, ps);
                if (ps >= (uint32_t)kEndPosModelIndex) pr += (((ps >> 1) - 1) - kNumAlignBits) << 6;
                psp[st + ps] = (uint16_t)pr;
            }
        }
        LANE_FENCE();
        for (uint32_t l = 0; l < (uint32_t)kNumLenToPosStates; l++) {
            uint32_t st = l << kNumPosSlotBits, st2 = l * kNumFullDistances;
            LANE_FOR(uint32_t, i, 0u, (uint32_t)kNumFullDistances)
                dp[st2 + i] = (uint16_t)(i < (uint32_t)kStartPosModelIndex ? psp[st + i] : psp[st + pos_slot(i)] + tp[i]);
        }
        match_price_count = 0;
        LANE_FENCE();
    }
    FI void fill_align_prices() {   // Encoder.java:1120-1125
        LANE_FOR(uint32_t, i, 0u, (uint32_t)kAlignTableSize) ap[i] = rev_price(probs + E_ALIGN, kNumAlignBits, i);
        align_price_count = 0;
        LANE_FENCE();
    }

    // ------------------------------------------------------------ match lists (phase 1 output)
    FI void ring_fill(uint32_t base) {
        ring_base = base;
        LANE_FOR(uint32_t, k, 0u, (uint32_t)kRing) {
            const uint32_t e = k;
            uint32_t q = base + k;
            uint32_t info = 0;
            PairT p0 = 0, p1 = 0, p2 = 0, p3 = 0;
            if (q < n) {
                uint64_t g0 = gbase + q;
                // streamed once: non-temporal, so they do not evict the literal models from L2
                PairT q[kInlinePairs];
                info = load_rec<PairT>(pairs + g0 * rec_vecs<PairT>(), q);
                p0 = q[0]; p1 = q[1]; p2 = q[2]; p3 = q[3];
            }
            ring_info[e] = info;
            PairT* dst = ring_pairs + e * kInlinePairs;
            dst[0] = p0; dst[1] = p1; dst[2] = p2; dst[3] = p3;
        }
        LANE_FENCE();
    }
    FI uint32_t read_match_distances() {   // Encoder.ReadMatchDistances (Encoder.java:275-287), extension precomputed
        PBEGIN(t0);
        uint32_t q = mfpos;
        if (q - ring_base >= (uint32_t)kRing) ring_fill(q);
        const uint32_t slot = q - ring_base;
        uint32_t info = ring_info[slot];
        uint32_t cnt = info & 0xFFFFu, ml = info >> 16;
        if (cnt <= (uint32_t)kInlinePairs) {   // read in place from the ring: no copy, no LDS round trip
            mdp = ring_pairs + slot * kInlinePairs;
        } else {
            PCOUNT(PF_NOVF);
            LANE_FOR(uint32_t, k, 0u, cnt)
                md_buf[k] = k < (uint32_t)kInlinePairs ? ring_pairs[slot * kInlinePairs + k]
                                                       : ovf[(uint64_t)ovf_off[gbase + q] * ovf_stride(fb) + k - kInlinePairs];
            LANE_FENCE();
            mdp = md_buf;
        }
        num_pairs = cnt;
        mfpos++;
        additional_offset++;
        PEND(PF_MATCHES, t0);
        return ml;
    }
    FI void move_pos(uint32_t num) {
        if (num > 0) { mfpos += num; additional_offset += (int32_t)num; }
    }
    FI uint32_t rep_len1_price(uint32_t st, uint32_t ps) const {
        return dm0(E_G0 + st) + dm0(E_R0L + (st << PBS) + ps);
    }
    FI uint32_t pure_rep_price(uint32_t ri, uint32_t st, uint32_t ps) const {
        uint32_t price;
        if (ri == 0) {
            price = dm0(E_G0 + st);
            price += dm1(E_R0L + (st << PBS) + ps);
        } else {
            price = dm1(E_G0 + st);
            if (ri == 1) price += dm0(E_G1 + st);
            else { price += dm1(E_G1 + st); price += dmb(E_G2 + st, ri - 2); }
        }
        return price;
    }
    FI uint32_t rep_price(uint32_t ri, uint32_t len, uint32_t st, uint32_t ps) const {
        return len_price(1, len - kMatchMinLen, ps) + pure_rep_price(ri, st, ps);
    }
    FI uint32_t dist_price(uint32_t pos, uint32_t len) const {   // GetPosLenPrice without the length part
        uint32_t lps = len_to_pos_state(len);
        if (pos < (uint32_t)kNumFullDistances) return (uint32_t)dp[lps * kNumFullDistances + pos];
        return (uint32_t)psp[(lps << kNumPosSlotBits) + pos_slot(pos)] + ap[pos & kAlignMask];
    }
    FI uint32_t pos_len_price(uint32_t pos, uint32_t len, uint32_t ps) const {   // Encoder.java:323-333
        return dist_price(pos, len) + len_price(0, len - kMatchMinLen, ps);
    }
    // while (lenEnd < target) _optimum[++lenEnd].Price = kIfinityPrice
    FI void extend_to(uint32_t& len_end, uint32_t target, uint32_t cur) {
        if (len_end >= target) return;
        if (RING) {
            if (target > cur + (uint32_t)kOptLds + 1) { bad = 8; return; }   // beyond cur + 2 fb + 1
            uint32_t hi = target;
            if (hi > cur + (uint32_t)kOptLds) {   // cur + 65: its entry still holds cur + 1
                far_valid = 1;
                o_price[kFarEntry] = kInfinityPrice; o_pp[kFarEntry] = 0; o_bp[kFarEntry] = 0; o_bp2[kFarEntry] = 0;
                hi--;
            }
            if (hi >= (uint32_t)kOptLds) {   // entries reused: write back slots i - 64 first
                LANE_FOR(uint32_t, i, len_end + 1, hi + 1) {
                    const uint32_t r = i & kOptMask;
                    if (i >= (uint32_t)kOptLds) {
                        const uint32_t h = i - (uint32_t)kOptLds;
                        sstore(1, h, o_pp[r]); sstore(2, h, (uint32_t)o_bp[r]); sstore(3, h, (uint32_t)o_bp2[r]);
                    }
                    o_price[r] = kInfinityPrice;
                }
            } else {
                for (uint32_t i0 = len_end + 1; i0 <= hi; i0 += kWave) {
                    const uint32_t i = i0 + lane_id();
                    o_price[i <= hi ? i : (uint32_t)kOptLds] = kInfinityPrice;
                }
            }
            if (hi > ring_top) ring_top = hi;
            len_end = target;
            LANE_FENCE();
            return;
        }
        if (target < (uint32_t)kOptLds) {   // branch-free: idle lanes write the sink slot
            for (uint32_t i0 = len_end + 1; i0 <= target; i0 += kWave) {
                const uint32_t i = i0 + lane_id();
                o_price[i <= target ? i : (uint32_t)kOptLds] = kInfinityPrice;
            }
            len_end = target;
            LANE_FENCE();
            return;
        }
        LANE_FOR(uint32_t, i, len_end + 1, target + 1) set_price(i, kInfinityPrice);
        len_end = target;
        fence_upto(target);
    }
    // lanes relax slots base+l, l in [lo, hi], with a rep of index ri
    FI void relax_rep(uint32_t base_slot, uint32_t lo, uint32_t hi, uint32_t price_base, uint32_t ps,
                      uint32_t pos_prev_v, uint32_t ri) {
        if (RING || base_slot + hi < (uint32_t)kOptLds) {   // all slots in LDS: no per-lane spill branches
            // branch-free: idle lanes and lanes that do not improve write the sink slot
            for (uint32_t l0 = lo; l0 <= hi; l0 += kWave) {
                const uint32_t l = l0 + lane_id();
                const bool ok = l <= hi;
                const uint32_t s = ok ? ix(base_slot + l) : (uint32_t)kOptLds;
                const uint32_t cl = price_base + len_price(1, ok ? l - 2 : 0u, ps);
                const uint32_t t = (ok && cl < o_price[s]) ? s : (uint32_t)kOptLds;
                o_price[t] = cl;
                o_pp[t] = pos_prev_v;   // Prev1IsChar = false (PosPrev2 / Prev2 are read only with it)
                o_bp[t] = (int32_t)ri;
            }
            LANE_FENCE();
            return;
        }
        LANE_FOR(uint32_t, l, lo, hi + 1) {
            uint32_t cl = price_base + len_price(1, l - 2, ps);
            uint32_t s = base_slot + l;
            if (cl < price_at(s)) {
                set_price(s, cl);
                set_pp(s, pos_prev_v);
                set_bp(s, (int32_t)ri);
            }
        }
        fence_upto(base_slot + hi);
    }
    // lanes relax slots base+l, l in [lo, hi], all with the match distance `dist`
    FI void relax_match(uint32_t base_slot, uint32_t lo, uint32_t hi, uint32_t price_base, uint32_t dist, uint32_t ps,
                        uint32_t pos_prev_v) {
        if (RING || base_slot + hi < (uint32_t)kOptLds) {   // all slots in LDS; branch-free as relax_rep
            for (uint32_t l0 = lo; l0 <= hi; l0 += kWave) {
                const uint32_t l = l0 + lane_id();
                const bool ok = l <= hi;
                const uint32_t s = ok ? ix(base_slot + l) : (uint32_t)kOptLds;
                const uint32_t cl = price_base + pos_len_price(dist, ok ? l : (uint32_t)kMatchMinLen, ps);
                const uint32_t t = (ok && cl < o_price[s]) ? s : (uint32_t)kOptLds;
                o_price[t] = cl;
                o_pp[t] = pos_prev_v;
                o_bp[t] = (int32_t)(dist + kNumRepDistances);
            }
            LANE_FENCE();
            return;
        }
        LANE_FOR(uint32_t, l, lo, hi + 1) {
            uint32_t cl = price_base + pos_len_price(dist, l, ps);
            uint32_t s = base_slot + l;
            if (cl < price_at(s)) {
                set_price(s, cl);
                set_pp(s, pos_prev_v);
                set_bp(s, (int32_t)(dist + kNumRepDistances));
            }
        }
        fence_upto(base_slot + hi);
    }
    // getOptimum's match candidates of position 0 (Encoder.java:620-640)
    template <bool F>
    FI void relax_first(uint32_t lstart, uint32_t len_main, uint32_t npairs, uint32_t normal_match_price, uint32_t pos_state) {
        if (F) {   // all slots in LDS: branch-free (idle and non-improving lanes write the sink slot)
            for (uint32_t l0 = lstart; l0 <= len_main; l0 += kWave) {
                const uint32_t l = l0 + lane_id();
                const bool ok = l <= len_main;
                // the pair of length l: the first with md_len >= l (lengths increase), i.e. the count of
                // shorter ones among the first npairs - 1 -- a uniform loop instead of a per-lane while
                uint32_t k = 0;
                for (uint32_t kk = 0; kk + 1 < npairs; kk++) k += l > md_l(kk) ? 1u : 0u;
                const uint32_t distance = md_d(k);
                const uint32_t s = ok ? l : (uint32_t)kOptLds;
                const uint32_t cl = normal_match_price + pos_len_price(distance, ok ? l : (uint32_t)kMatchMinLen, pos_state);
                const uint32_t t = (ok && cl < o_price[s]) ? s : (uint32_t)kOptLds;
                o_price[t] = cl;
                o_pp[t] = 0u;
                o_bp[t] = (int32_t)(distance + kNumRepDistances);
            }
            LANE_FENCE();
            return;
        }
        LANE_FOR(uint32_t, l, lstart, len_main + 1) {
            uint32_t k = 0;
            while (k + 1 < npairs && l > md_l(k)) k++;
            uint32_t distance = md_d(k);
            uint32_t cl = normal_match_price + pos_len_price(distance, l, pos_state);
            if (cl < price_at<F>(l)) {
                set_price<F>(l, cl);
                set_pp<F>(l, 0u);
                set_bp<F>(l, (int32_t)(distance + kNumRepDistances));
            }
        }
        if (F) LANE_FENCE(); else fence_upto(len_main);
    }
    // uniform single-slot update for the two-step (x + literal + rep0) candidates
    template <bool F> FI void relax_two_step_t(uint32_t s, uint32_t cl, uint32_t pos_prev_v, bool prev2, uint32_t pos_prev2_v, int32_t back2) {
        if (cl < price_at<F>(s)) {
            set_price<F>(s, cl);
            set_bp<F>(s, 0);
            if (prev2) {
                set_pp<F>(s, pos_prev_v | (pos_prev2_v << kPos2Shift) | (3u << kFlagShift));
                set_bp2<F>(s, back2);
            } else {
                set_pp<F>(s, pos_prev_v | (1u << kFlagShift));
            }
        }
        fence_upto(s);
    }

    FI void relax_two_step(uint32_t s, uint32_t cl, uint32_t pos_prev_v, bool prev2, uint32_t pos_prev2_v, int32_t back2,
                           uint32_t cur) {
        PCOUNT(PF_NTWO);
        if (RING) {
            if (far_valid && s == cur + (uint32_t)kOptLds + 1) {   // slot cur + 65: the far entry
                const uint32_t e = kFarEntry;
                if (cl < o_price[e]) {
                    o_price[e] = cl;
                    o_bp[e] = 0;
                    if (prev2) { o_pp[e] = pos_prev_v | (pos_prev2_v << kPos2Shift) | (3u << kFlagShift); o_bp2[e] = back2; }
                    else o_pp[e] = pos_prev_v | (1u << kFlagShift);
                }
                LANE_FENCE();
                return;
            }
            relax_two_step_t<true>(s, cl, pos_prev_v, prev2, pos_prev2_v, back2);
            return;
        }
        if (s < (uint32_t)kOptLds) relax_two_step_t<true>(s, cl, pos_prev_v, prev2, pos_prev2_v, back2);
        else relax_two_step_t<false>(s, cl, pos_prev_v, prev2, pos_prev2_v, back2);
    }

    template <bool F> FI uint32_t backward_t(int32_t* back_res, uint32_t cur) {   // Encoder.java:335-362
        PBEGIN(tb);
        opt_end = (int32_t)cur;
        uint32_t pos_mem = pos_prev<F>(cur);
        int32_t back_mem = bp_at<F>(cur);
        uint32_t guard = 0;
        do {
            if (++guard > (uint32_t)kNumOpts || pos_mem >= cur) { bad = 2; break; }
            uint32_t fsc = fs_at<F>(cur);
            if (fsc & 1u) {
                set_bp<F>(pos_mem, -1);
                set_pp<F>(pos_mem, pos_mem - 1);   // MakeAsChar (Optimal.java:22-25): flags cleared
                if (fsc & 2u) {
                    uint32_t m1 = pos_mem - 1;
                    set_pp<F>(m1, pos_prev2<F>(cur));
                    set_bp<F>(m1, bp2_at<F>(cur));
                }
            }
            uint32_t ppv = pos_mem;
            int32_t back_cur = back_mem;
            back_mem = bp_at<F>(ppv);
            pos_mem = pos_prev<F>(ppv);
            set_bp<F>(ppv, back_cur);
            set_pp<F>(ppv, (pp_at<F>(ppv) & ~kPosMask) | cur);   // PosPrev = cur; ppv's flags stay
            cur = ppv;
        } while (cur > 0);
        opt_cur = (int32_t)pos_prev<F>(0);
        *back_res = bp_at<F>(0);
        PEND(PF_BACK, tb);
        return (uint32_t)opt_cur;
    }

    FI uint32_t backward(int32_t* back_res, uint32_t cur) {   // every slot touched is <= cur
        if (RING) {
            if (ring_top < (uint32_t)kOptLds) return backward_t<true>(back_res, cur);
            SPILL_FENCE();   // the write-backs before the home reads
            const uint32_t r = backward_t<false>(back_res, cur);
            SPILL_FENCE();   // and Backward's home writes before the cached path reads them
            return r;
        }
        return cur < (uint32_t)kOptLds ? backward_t<true>(back_res, cur) : backward_t<false>(back_res, cur);
    }

    // getOptimum (Encoder.java:364-811). Returns length; *back_res = pos.
    FI uint32_t get_optimum(uint32_t position, int32_t* back_res, uint32_t* sym_slot) {
        if (opt_end != opt_cur) {
            uint32_t c = (uint32_t)opt_cur;
            *sym_slot = c;
            uint32_t nxt;
            if (a_in(c)) { nxt = pos_prev<true>(c); *back_res = bp_at<true>(c); }
            else { nxt = pos_prev(c); *back_res = bp_at(c); }
            opt_cur = (int32_t)nxt;
            if (nxt <= c || nxt > (uint32_t)opt_end) { bad = 3; return 1; }
            return nxt - c;
        }
        opt_cur = opt_end = 0;
        *sym_slot = 0;
        if (RING) { ring_top = 0; far_valid = 0; }
        uint32_t len_main;
        if (longest_found) { len_main = longest_len; longest_found = 0; }
        else len_main = read_match_distances();
        uint32_t npairs = num_pairs;
        rp0 = rd0; rp1 = rd1; rp2 = rd2; rp3 = rd3;
        PCOUNT(PF_NOPT);
        PBEGIN(t0);
        gather(false);
        set_bytes<true>(0, win_bytes() | (state << 24));
        uint32_t num_avail = avail() + 1;
        if (num_avail < 2) { *back_res = -1; LANE_FENCE(); return 1; }
        if (num_avail > (uint32_t)kMatchMaxLen) num_avail = kMatchMaxLen;
        // a rep whose first byte differs (offset 0's mask bit clear) has length 0: no glen
        uint32_t rl0 = eq1(gm0, 0) ? glen(gm0, rp0, 0, kMatchMaxLen) : 0u;
        uint32_t rl1 = eq1(gm1, 0) ? glen(gm1, rp1, 0, kMatchMaxLen) : 0u;
        uint32_t rl2 = eq1(gm2, 0) ? glen(gm2, rp2, 0, kMatchMaxLen) : 0u;
        uint32_t rl3 = eq1(gm3, 0) ? glen(gm3, rp3, 0, kMatchMaxLen) : 0u;
        PEND(PF_REPLEN, t0);
        uint32_t rep_max = 0, rl_max = rl0;
        if (rl1 > rl_max) { rep_max = 1; rl_max = rl1; }
        if (rl2 > rl_max) { rep_max = 2; rl_max = rl2; }
        if (rl3 > rl_max) { rep_max = 3; rl_max = rl3; }
        if (rl_max >= fb) {
            *back_res = (int32_t)rep_max;
            move_pos(rl_max - 1);
            return rl_max;
        }
        if (len_main >= fb) {
            *back_res = (int32_t)(md_d(npairs - 1) + kNumRepDistances);
            move_pos(len_main - 1);
            return len_main;
        }
        uint32_t cur_byte = g_cur;
        uint32_t match_byte = g_mb;   // rp0 == rd0 here
        if (len_main < 2 && cur_byte != match_byte && rl_max < 2) { *back_res = -1; return 1; }

        uint32_t pos_state = position & ps_mask;
        PBEGIN(t1);
        uint32_t p1 = dm0(E_IS_MATCH + (state << PBS) + pos_state) +
                      lit_price(lit_coder(position, g_prev), !st_is_char(state), match_byte, cur_byte);
        PEND(PF_LIT, t1);
        uint32_t match_price = dm1(E_IS_MATCH + (state << PBS) + pos_state);
        uint32_t rep_match_price = match_price + dm1(E_IS_REP + state);
        int32_t bp1 = -1;
        if (match_byte == cur_byte) {
            uint32_t srp = rep_match_price + rep_len1_price(state, pos_state);
            if (srp < p1) { p1 = srp; bp1 = 0; }
        }
        set_price<true>(1, p1);
        set_bp<true>(1, bp1);
        uint32_t len_end = len_main >= rl_max ? len_main : rl_max;
        if (len_end < 2) { *back_res = bp1; LANE_FENCE(); return 1; }
        set_pp<true>(1, 0u);
        set_backs4<true>(0, rp0, rp1, rp2, rp3);
        LANE_FENCE();
        PBEGIN(t2);
        if (len_end < (uint32_t)kOptLds) {
            LANE_FOR(uint32_t, l, 2u, len_end + 1) set_price<true>(l, kInfinityPrice);
            if (RING) ring_top = len_end;
            LANE_FENCE();
        } else {
            LANE_FOR(uint32_t, l, 2u, len_end + 1) set_price(l, kInfinityPrice);
            fence_upto(len_end);
        }
#pragma unroll
        for (uint32_t i = 0; i < (uint32_t)kNumRepDistances; i++) {
            uint32_t rl = sel4(i, rl0, rl1, rl2, rl3);
            if (rl < 2) continue;
            relax_rep(0, 2, rl, rep_match_price + pure_rep_price(i, state, pos_state), pos_state, 0, i);
        }
        uint32_t normal_match_price = match_price + dm0(E_IS_REP + state);
        uint32_t lstart = rl0 >= 2 ? rl0 + 1 : 2;
        if (lstart <= len_main) {
            // no look-ahead in this loop: every length is independent
            if (len_main < (uint32_t)kOptLds) relax_first<true>(lstart, len_main, npairs, normal_match_price, pos_state);
            else relax_first<false>(lstart, len_main, npairs, normal_match_price, pos_state);
        }
        PEND(PF_RELAX, t2);
        return parse_forward(position, back_res, len_end);
    }

    // Position step of getOptimum's forward loop (Encoder.java:685-742): the state
    // and reps of cur from its best path, the literal and short-rep candidates
    // of cur + 1. F: every slot touched (<= cur + 1) is below kOptLds, so the
    // slot accesses are plain LDS operations (no spill branches, and no wait on
    // outstanding HBM operations merged into them).
    // It is two parts: S (pos_state_part: the state, the reps, the gather and the literal
    // price of cur; reads slot cur and its predecessors, all final) and N (pos_next_part:
    // the literal / short-rep update of slot cur + 1, which cur - 1's longer candidates may
    // have written).
    struct PosS { uint32_t st, pos_state, cur_price, cur_and1, cur_byte, match_byte; };
#ifndef LZG_VSEL_STATE
#define LZG_VSEL_STATE 2
#endif
    static constexpr bool kVselState = LZG_VSEL_STATE == 2 ? true : (LZG_VSEL_STATE == 1 ? !LIT_LDS : false);
    template <bool F>
    FI PosS pos_state_part(uint32_t cur, uint32_t position) {
        PBEGIN(ts);
        // F: cur + 1 < kOptLds, every slot touched is in LDS. RING deep steps: the
        // ahead fields of cur and cur + 1 are in the ring (FA); the behind fields of
        // the predecessor may be in HBM (a path back by 65), checked per access.
        constexpr bool FA = F || RING, FB = F;
        PosS r;
        if constexpr (F && kVselState) {
            // Branch-free form (the many-streams kernel, where the vector unit is idle and the
            // scalar unit is the shared resource): the derivation below as mask arithmetic on the
            // LDS-loaded values (bit operations the compiler cannot turn back into branches), with
            // one 16-byte Backs read whether or not it is needed. The State transitions (Base.java
            // :16-36) as packed 4-bit tables / closed forms: match 7 | 10, long 8 | 11, short 9 | 11.
            constexpr uint64_t kLitT = 0x54654321'0000ull;   // st_lit: 0 0 0 0 1 2 3 4 5 6 4 5
            const uint32_t ppc = pp_at<true>(cur);
            const uint32_t bpc = (uint32_t)bp_at<true>(cur), bp2c = (uint32_t)bp2_at<true>(cur);
            const uint32_t c1 = (ppc >> kFlagShift) & 1u;                                // Prev1IsChar
            const uint32_t c2 = (ppc >> (kFlagShift + 1)) & c1;                          // and Prev2
            const uint32_t m2 = 0u - c2;
            const uint32_t pp2 = (ppc >> kPos2Shift) & kPosMask;
            const uint32_t pprev = (ppc & kPosMask) - c1;
            const uint32_t q = pprev ^ ((pp2 ^ pprev) & m2);   // the slot of the start state and of the Backs
            const uint32_t mlit = 0u - (uint32_t)(pprev == cur - 1);   // a literal / short rep from cur - 1
            const uint32_t st0 = state_at<true>(q, cur - 1);
            const v4u32 b = backs4_at<true>(q, cur - 1);
            const uint32_t pos = bpc ^ ((bp2c ^ bpc) & m2);   // the last symbol's back (int32 as bits)
            const uint32_t rep_pos = (uint32_t)((int32_t)pos < kNumRepDistances);
            // st1: after the Prev2 symbol (long rep or match), st2: after the middle literal
            const uint32_t a1 = 7u + 3u * (uint32_t)(st0 >= 7u) + (uint32_t)((int32_t)bp2c < kNumRepDistances);
            const uint32_t st1 = st0 ^ ((a1 ^ st0) & m2);
            const uint32_t l2 = (uint32_t)(kLitT >> (4u * st1)) & 15u;
            const uint32_t st2 = st1 ^ ((l2 ^ st1) & (0u - c1));
            const uint32_t hi2 = (uint32_t)(st2 >= 7u);
            const uint32_t lit_st = bpc == 0u ? 9u + 2u * hi2 : ((uint32_t)(kLitT >> (4u * st2)) & 15u);
            const uint32_t far_st = 7u + 3u * hi2 + (c2 | rep_pos);
            const uint32_t st = far_st ^ ((lit_st ^ far_st) & mlit);
            // the reps: a rep r moves Backs[r] to the front, a match shifts its distance in
            const uint32_t r3 = pos < 3u ? pos : 3u;   // (as unsigned: a match, and -1, give 3)
            const uint32_t b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3];
            const uint32_t e0 = 0u - (uint32_t)(r3 == 0u), e1 = 0u - (uint32_t)(r3 == 1u), e2 = 0u - (uint32_t)(r3 == 2u);
            const uint32_t br = (b0 & e0) | (b1 & e1) | (b2 & e2) | (b3 & ~(e0 | e1 | e2));
            const uint32_t n0 = rep_pos ? br : pos - (uint32_t)kNumRepDistances;
            const uint32_t n1 = b0 ^ ((b1 ^ b0) & e0);
            const uint32_t n2 = b1 ^ ((b2 ^ b1) & (e0 | e1));
            const uint32_t n3 = b2 ^ ((b3 ^ b2) & ~(0u - (uint32_t)(r3 == 3u)));
            rp0 = n0 ^ ((rp0 ^ n0) & mlit);
            rp1 = n1 ^ ((rp1 ^ n1) & mlit);
            rp2 = n2 ^ ((rp2 ^ n2) & mlit);
            rp3 = n3 ^ ((rp3 ^ n3) & mlit);
            set_backs4<true>(cur, rp0, rp1, rp2, rp3);
            r.cur_price = price_at<true>(cur);
            r.pos_state = position & ps_mask;
            r.st = st;
            PEND(PF_STATE, ts);
            return r;
        }
        uint32_t st;
        uint32_t ppc = pp_at<FA>(cur);
        uint32_t pos_prev_c = ppc & kPosMask;
        uint32_t fsc = ppc >> kFlagShift;
        int32_t bpc = bp_at<FA>(cur);
        uint32_t pprev = pos_prev_c;
        if (fsc & 1u) {
            pprev--;
            if (fsc & 2u) {
                st = state_at<FB>((ppc >> kPos2Shift) & kPosMask, cur - 1);
                if (bp2_at<FA>(cur) < kNumRepDistances) st = st_long(st);
                else st = st_match(st);
            } else st = state_at<FB>(pprev, cur - 1);
            st = st_lit(st);
        } else st = state_at<FB>(pprev, cur - 1);
        if (pprev == cur - 1) {
            if (bpc == 0) st = st_short(st);
            else st = st_lit(st);
        } else {
            int32_t pos;
            if ((fsc & 1u) && (fsc & 2u)) {
                pprev = (ppc >> kPos2Shift) & kPosMask;
                pos = bp2_at<FA>(cur);
                st = st_long(st);
            } else {
                pos = bpc;
                if (pos < kNumRepDistances) st = st_long(st);
                else st = st_match(st);
            }
            const v4u32 b = backs4_at<FB>(pprev, cur - 1);
            const uint32_t b0 = b[0], b1 = b[1], b2 = b[2], b3 = b[3];
            if (pos < kNumRepDistances) {
                if (pos == 0) { rp0 = b0; rp1 = b1; rp2 = b2; rp3 = b3; }
                else if (pos == 1) { rp0 = b1; rp1 = b0; rp2 = b2; rp3 = b3; }
                else if (pos == 2) { rp0 = b2; rp1 = b0; rp2 = b1; rp3 = b3; }
                else { rp0 = b3; rp1 = b0; rp2 = b1; rp3 = b2; }
            } else {
                rp0 = (uint32_t)(pos - kNumRepDistances); rp1 = b0; rp2 = b1; rp3 = b2;
            }
        }
        if (RING) {   // cur's entry held cur - 64
            if (!F && cur >= (uint32_t)kOptLds) evict_behind(cur - (uint32_t)kOptLds);
        }
        set_backs4<FA>(cur, rp0, rp1, rp2, rp3);
        r.cur_price = price_at<FA>(cur);
        r.pos_state = position & ps_mask;
        r.st = st;
        PEND(PF_STATE, ts);
        return r;
    }
    template <bool F>
    FI void pos_gather_part(uint32_t cur, uint32_t position, PosS& r) {
        constexpr bool FA = F || RING;
        PBEGIN(tg);
        gather(true);
        set_bytes<FA>(cur, win_bytes() | (r.st << 24));
        PEND(PF_REPLEN, tg);
        r.cur_byte = g_cur;
        r.match_byte = g_mb;
        PBEGIN(tl);
        r.cur_and1 = r.cur_price + dm0(E_IS_MATCH + (r.st << PBS) + r.pos_state) +
                     lit_price(lit_coder(position, g_prev), !st_is_char(r.st), r.match_byte, r.cur_byte);
        PEND(PF_LIT, tl);
    }
    // N: slot cur + 1's literal and short-rep candidates (nx_*: its fields, read by the caller)
    template <bool F>
    FI bool pos_next_part(uint32_t cur, const PosS& r, uint32_t nx_price, uint32_t nx_pp, int32_t nx_bp,
                          uint32_t& match_price, uint32_t& rep_match_price) {
        constexpr bool FA = F || RING;
        PBEGIN(tn);
        const uint32_t nx = cur + 1, st = r.st, pos_state = r.pos_state;
        bool next_is_char = false;
        if (r.cur_and1 < nx_price) {
            nx_price = r.cur_and1; nx_pp = cur; nx_bp = -1;
            set_price<FA>(nx, nx_price); set_pp<FA>(nx, nx_pp); set_bp<FA>(nx, -1);
            next_is_char = true;
        }
        match_price = r.cur_price + dm1(E_IS_MATCH + (st << PBS) + pos_state);
        rep_match_price = match_price + dm1(E_IS_REP + st);
        if (r.match_byte == r.cur_byte && !((nx_pp & kPosMask) < cur && nx_bp == 0)) {
            uint32_t srp = rep_match_price + rep_len1_price(st, pos_state);
            if (srp <= nx_price) {
                set_price<FA>(nx, srp); set_pp<FA>(nx, cur); set_bp<FA>(nx, 0);
                next_is_char = true;
            }
        }
        fence_upto(nx);
        PEND(PF_STATE, tn);
        return next_is_char;
    }
    template <bool F>
    FI bool pos_step(uint32_t cur, uint32_t position, PosS& r, uint32_t& match_price, uint32_t& rep_match_price) {
        constexpr bool FA = F || RING;
        r = pos_state_part<F>(cur, position);
        // cur + 1's slot: nothing before its literal / short-rep update below writes it, so its
        // reads are issued before the gather and complete under the gather's memory round trip
        const uint32_t nx = cur + 1;
        const uint32_t nx_price = price_at<FA>(nx), nx_pp = pp_at<FA>(nx);
        const int32_t nx_bp = bp_at<FA>(nx);
        pos_gather_part<F>(cur, position, r);
        return pos_next_part<F>(cur, r, nx_price, nx_pp, nx_bp, match_price, rep_match_price);
    }

    // R: the rest of position cur's step (Encoder.java:743-808): the literal + rep0
    // look-ahead, the rep candidates and the match candidates with their two-step
    // look-aheads, relaxing slots >= cur + 2 (len_end grows with them).
    FI void relax_step(uint32_t cur, uint32_t position, const PosS& r, bool next_is_char, uint32_t match_price,
                       uint32_t rep_match_price, uint32_t new_len, uint32_t npairs, uint32_t& len_end) {
        const uint32_t st = r.st, pos_state = r.pos_state, cur_and1 = r.cur_and1;
        const uint32_t match_byte = r.match_byte, cur_byte = r.cur_byte;
        if (RING && far_valid) {   // slot cur + 64 leaves the far entry for cur's, free now
            evict_ahead(cur);
            const uint32_t rr = cur & kOptMask, e = kFarEntry;
            const uint32_t fp = o_price[e], fpp = o_pp[e];
            const int32_t fbp = o_bp[e], fbp2 = o_bp2[e];
            o_price[rr] = fp; o_pp[rr] = fpp; o_bp[rr] = fbp; o_bp2[rr] = fbp2;
            ring_top = cur + (uint32_t)kOptLds;
            far_valid = 0;
            LANE_FENCE();
        }
        uint32_t num_avail_full = avail() + 1;
        if ((uint32_t)kNumOpts - 1 - cur < num_avail_full) num_avail_full = kNumOpts - 1 - cur;
        uint32_t num_avail = num_avail_full;
        if (num_avail < 2) return;
        if (num_avail > fb) num_avail = fb;
        // literal + rep0: lenTest2 >= 2 needs the bytes at offsets 1 and 2 equal
        if (!next_is_char && match_byte != cur_byte && eq2(gm0, 1)) {
            uint32_t t = num_avail_full - 1 < fb ? num_avail_full - 1 : fb;
            PBEGIN(t2a);
            uint32_t lt2 = glen(gm0, rp0, 1, (int32_t)t);
            PEND(PF_TWOLEN, t2a);
            if (lt2 >= 2) {
                PBEGIN(t2b);
                uint32_t st2 = st_lit(st);
                uint32_t psn = (position + 1) & ps_mask;
                uint32_t nrmp = cur_and1 + dm1(E_IS_MATCH + (st2 << PBS) + psn) + dm1(E_IS_REP + st2);
                uint32_t offset = cur + 1 + lt2;
                extend_to(len_end, offset, cur);
                relax_two_step(offset, nrmp + rep_price(0, lt2, st2, psn), cur + 1, false, 0, 0, cur);
                PEND(PF_RELAX, t2b);
            }
        }
        uint32_t start_len = 2;
#pragma unroll
        for (uint32_t ri = 0; ri < (uint32_t)kNumRepDistances; ri++) {
            uint32_t rdist = sel4(ri, rp0, rp1, rp2, rp3);
            const GM gmr = ri == 0 ? gm0 : (ri == 1 ? gm1 : (ri == 2 ? gm2 : gm3));
            // lenTest >= 2 needs offsets 0 and 1 equal: most reps stop here
            if (!eq2(gmr, 0)) continue;
            PBEGIN(tr);
            uint32_t lt = glen(gmr, rdist, 0, (int32_t)num_avail);
            PEND(PF_REPLEN, tr);
            if (lt < 2) continue;
            PBEGIN(trr);
            extend_to(len_end, cur + lt, cur);
            relax_rep(cur, 2, lt, rep_match_price + pure_rep_price(ri, st, pos_state), pos_state, cur, ri);
            PEND(PF_RELAX, trr);
            if (ri == 0) start_len = lt + 1;
            // the two-step lenTest2 >= 2 needs offsets lt + 1 and lt + 2 equal
            if (lt < num_avail_full && eq2(gmr, lt + 1)) {
                uint32_t t = num_avail_full - 1 - lt;
                if (t > fb) t = fb;
                PBEGIN(tq);
                uint32_t lt2 = glen(gmr, rdist, (int32_t)lt + 1, (int32_t)t);
                PEND(PF_TWOLEN, tq);
                if (lt2 >= 2) {
                    PBEGIN(tq2);
                    uint32_t st2 = st_long(st);
                    uint32_t psn = (position + lt) & ps_mask;
                    uint32_t clcp = rep_match_price + rep_price(ri, lt, st, pos_state) +
                                    dm0(E_IS_MATCH + (st2 << PBS) + psn) +
                                    lit_price(lit_coder(position + lt, a_byte((int32_t)lt - 1)), true,
                                              b_byte(1 + (int)ri, rdist, (int32_t)lt), a_byte((int32_t)lt));
                    st2 = st_lit(st2);
                    psn = (position + lt + 1) & ps_mask;
                    uint32_t nrmp = clcp + dm1(E_IS_MATCH + (st2 << PBS) + psn) + dm1(E_IS_REP + st2);
                    uint32_t offset = lt + 1 + lt2;
                    extend_to(len_end, cur + offset, cur);
                    relax_two_step(cur + offset, nrmp + rep_price(0, lt2, st2, psn), cur + lt + 1, true, cur, (int32_t)ri, cur);
                    PEND(PF_TWOREL, tq2);
                }
            }
        }
        if (new_len > num_avail) {
            new_len = num_avail;
            uint32_t np0 = npairs;
            for (npairs = 0; npairs + 1 < np0 && new_len > md_l(npairs); npairs++) {}
            // the clamped list goes to md_buf (the ring slot stays the match finder's)
            LANE_FOR(uint32_t, k, 0u, npairs + 1)
                md_buf[k] = k < npairs ? mdp[k] : PP::pack(new_len, md_d(npairs));
            LANE_FENCE();
            mdp = md_buf;
            npairs++;
        }
        if (new_len >= start_len) {
#ifdef LZG_PROF
            uint64_t tm = PCLK();
#endif
            uint32_t normal_match_price = match_price + dm0(E_IS_REP + st);
            extend_to(len_end, cur + new_len, cur);
            uint32_t offs = 0;
            while (offs + 1 < npairs && start_len > md_l(offs)) offs++;
            uint32_t seg_lo = start_len;
            for (uint32_t seg_guard = 0;; seg_guard++) {
#ifdef LZG_PROF
                if (seg_guard) tm = PCLK();
#endif
                if (seg_guard > (uint32_t)kMdCap || md_l(offs) < seg_lo) { bad = 6; break; }
                uint32_t seg_hi = md_l(offs);
                uint32_t cur_back = md_d(offs);
                relax_match(cur, seg_lo, seg_hi, normal_match_price, cur_back, pos_state, cur);
                PEND(PF_RELAX, tm);
                uint32_t lt = seg_hi;
                const int side = offs < 2 ? 5 + (int)offs : -1;
                const GM gmp = offs == 0 ? gmp0 : gmp1;
                if (lt < num_avail_full && (side < 0 || eq2(gmp, lt + 1))) {
                    uint32_t t = num_avail_full - 1 - lt;
                    if (t > fb) t = fb;
                    PBEGIN(tm2);
                    uint32_t lt2 = side > 0 ? glen(gmp, cur_back, (int32_t)lt + 1, (int32_t)t)
                                            : match_len((int32_t)lt, cur_back, (int32_t)t);
                    PEND(PF_TWOLEN, tm2);
                    if (lt2 >= 2) {
                        PBEGIN(tm3);
                        uint32_t cl = normal_match_price + pos_len_price(cur_back, lt, pos_state);
                        uint32_t st2 = st_match(st);
                        uint32_t psn = (position + lt) & ps_mask;
                        uint32_t clcp = cl + dm0(E_IS_MATCH + (st2 << PBS) + psn) +
                                        lit_price(lit_coder(position + lt, a_byte((int32_t)lt - 1)), true,
                                                  b_byte(side, cur_back, (int32_t)lt), a_byte((int32_t)lt));
                        st2 = st_lit(st2);
                        psn = (position + lt + 1) & ps_mask;
                        uint32_t nrmp = clcp + dm1(E_IS_MATCH + (st2 << PBS) + psn) + dm1(E_IS_REP + st2);
                        uint32_t offset = lt + 1 + lt2;
                        extend_to(len_end, cur + offset, cur);
                        relax_two_step(cur + offset, nrmp + rep_price(0, lt2, st2, psn), cur + lt + 1, true, cur,
                                       (int32_t)(cur_back + kNumRepDistances), cur);
                        PEND(PF_TWOREL, tm3);
                    }
                }
                offs++;
                if (offs == npairs) break;
                seg_lo = seg_hi + 1;
            }
        }
    }

    FI uint32_t parse_forward(uint32_t position, int32_t* back_res, uint32_t len_end) {
        uint32_t cur = 0;
        DBG(5, len_end);
        for (;;) {
            cur++;
            refresh_lane();
            DBG(6, cur);
            if (bad) { *back_res = -1; return 1; }
            if (cur == len_end) return backward(back_res, cur);
            if (cur >= (uint32_t)kNumOpts - 1 || len_end >= (uint32_t)kNumOpts) { bad = 4; *back_res = -1; return 1; }
            uint32_t new_len = read_match_distances();
            PCOUNT(PF_NPOS);
            uint32_t npairs = num_pairs;
            if (new_len >= fb) {
                longest_len = new_len;
                longest_found = 1;
                return backward(back_res, cur);
            }
            position++;
            PosS r;
            uint32_t match_price, rep_match_price;
            // every slot the step touches is <= cur + 1: LDS only when that is below kOptLds
#ifdef LZG_PROF
            if (cur + 1 >= (uint32_t)kOptLds) PCOUNT(PF_NSPILL);
#endif
            const bool next_is_char = cur + 1 < (uint32_t)kOptLds ? pos_step<true>(cur, position, r, match_price, rep_match_price)
                                                                   : pos_step<false>(cur, position, r, match_price, rep_match_price);
            relax_step(cur, position, r, next_is_char, match_price, rep_match_price, new_len, npairs, len_end);
        }
        __builtin_unreachable();   // the loop returns
    }

    // ------------------------------------------------------------ emitters (Encoder.java:860-1024, 818-841)
    // Codes one symbol: back = -1 literal (cb, match byte mb), 0..3 rep, >= 4 match
    // (distance back - 4); eos_marker codes WriteEndMarker's pseudo-match instead.
    FI void encode_symbol(int32_t back, uint32_t len, uint32_t now_pos, uint32_t cb, uint32_t mb, bool eos_marker) {
        Q q;
        q_init(q);
        const uint32_t ps = now_pos & ps_mask;
        int len_coder = -1;
        if (back == -1 && !eos_marker) {   // encodeSingleByteLiteral path (Encoder.java:893-903)
            q_bit(q, E_IS_MATCH + (state << PBS) + ps, 0);
            const uint32_t cidx = ((now_pos & ((1u << lp) - 1)) << lc) + (prev_byte >> (8 - lc));
            q_lit(q, cidx * 0x300u, !st_is_char(state), mb, cb);
            state = st_lit(state);
            prev_byte = cb;
        } else {
            q_bit(q, E_IS_MATCH + (state << PBS) + ps, 1);
            if (back >= 0 && back < kNumRepDistances && !eos_marker) {   // encodeARepetition (Encoder.java:938-974)
                q_bit(q, E_IS_REP + state, 1);
                if (back == 0) {
                    q_bit(q, E_G0 + state, 0);
                    q_bit(q, E_R0L + (state << PBS) + ps, len == 1 ? 0 : 1);
                } else {
                    q_bit(q, E_G0 + state, 1);
                    if (back == 1) q_bit(q, E_G1 + state, 0);
                    else { q_bit(q, E_G1 + state, 1); q_bit(q, E_G2 + state, (uint32_t)back - 2); }
                }
                if (len == 1) state = st_short(state);
                else { q_len(q, 1, len - kMatchMinLen, ps); len_coder = 1; state = st_long(state); }
                if (back == 1) { uint32_t t = rd1; rd1 = rd0; rd0 = t; }
                else if (back == 2) { uint32_t t = rd2; rd2 = rd1; rd1 = rd0; rd0 = t; }
                else if (back == 3) { uint32_t t = rd3; rd3 = rd2; rd2 = rd1; rd1 = rd0; rd0 = t; }
            } else {   // encodeAMatch (Encoder.java:976-1005); the end marker is the match
                       // (len 2, slot 63, reduced distance 2^30 - 1) of WriteEndMarker (:818-835)
                q_bit(q, E_IS_REP + state, 0);
                state = st_match(state);
                q_len(q, 0, len - kMatchMinLen, ps);
                len_coder = 0;
                const uint32_t pos = eos_marker ? 0xFFFFFFFFu : (uint32_t)(back - kNumRepDistances);
                const uint32_t slot = eos_marker ? 63u : pos_slot(pos);
                q_bt(q, E_PSLOT + (len_to_pos_state(len) << 6), kNumPosSlotBits, slot);
                if (slot >= (uint32_t)kStartPosModelIndex) {
                    const uint32_t footer = (slot >> 1) - 1, base = (2 | (slot & 1)) << footer, red = pos - base;
                    if (slot < (uint32_t)kEndPosModelIndex) q_rev(q, E_PENC + base - slot - 1, footer, red);
                    else {
                        q_direct(q, red >> kNumAlignBits, footer - kNumAlignBits);
                        q_rev(q, E_ALIGN, kNumAlignBits, red & kAlignMask);
                        align_price_count++;
                    }
                }
                rd3 = rd2; rd2 = rd1; rd1 = rd0; rd0 = pos;
                match_price_count++;
            }
            prev_byte = cb;   // the match's last byte
        }
        q_run(q, back == -1 && !eos_marker);
        if (len_coder >= 0) {   // LenPriceTableEncoder.Encode (LenPriceTableEncoder.java:31-37)
            const uint32_t c = lenc[len_coder * 16 + ps] - 1;
            lenc[len_coder * 16 + ps] = c;
            LANE_FENCE();
            if (c == 0) update_len_table(len_coder, ps);
        }
    }
    FI void flush(uint32_t now_pos) {   // the coder's own flush (5 x ShiftLow) runs in rc.hip
        if (eos) encode_symbol(0, kMatchMinLen, now_pos, prev_byte, 0, true);
        rec_store_tail();
        if constexpr (kSliced) save_state(now_pos, 1);   // the stream is done (the host reads SS_DONE)
    }

    // ------------------------------------------------------------ the sliced encode's state
    // (kSliced kernels; the layout is slice_layout). Every lane copies its share of each table;
    // the scalars go through one lane-indexed store per word (vector stores).
    FI uint32_t slice_scalar(uint32_t k, uint32_t now_pos, uint32_t done) const {
        const uint32_t v[SS_WORDS] = {kSliceMagic, now_pos, done, state, prev_byte, rd0, rd1, rd2, rd3,
                                      match_price_count, align_price_count, 0u, 0u, 0u, 0u, 0u};
        uint32_t r = 0;
#pragma unroll
        for (int i = 0; i < SS_WORDS; i++) r = k == (uint32_t)i ? v[i] : r;
        return r;
    }
    FI void save_state(uint32_t now_pos, uint32_t done) {
        uint32_t off[SL_COUNT];
        slice_layout(pb, lc, lp, tsize, off);
        const uint32_t nlit = 0x300u << (lc + lp);
        uint32_t* sc = (uint32_t*)(sst + off[SL_SCALARS]);
        LANE_FOR(uint32_t, k, 0u, (uint32_t)SS_WORDS) sc[k] = slice_scalar(k, now_pos, done);
        if (done) return;   // a finished stream needs no tables
        uint16_t* g16 = (uint16_t*)(sst + off[SL_PROBS]);
        LANE_FOR(uint32_t, i, 0u, (uint32_t)E_COUNT) g16[i] = probs[i];
        g16 = (uint16_t*)(sst + off[SL_LENP]);
        LANE_FOR(uint32_t, i, 0u, (2u << pb) * tsize) g16[i] = lenp[i];
        uint32_t* g32 = (uint32_t*)(sst + off[SL_LENC]);
        LANE_FOR(uint32_t, i, 0u, 32u) g32[i] = lenc[i];
        g16 = (uint16_t*)(sst + off[SL_PSP]);
        LANE_FOR(uint32_t, i, 0u, 256u) g16[i] = psp[i];
        g16 = (uint16_t*)(sst + off[SL_DP]);
        LANE_FOR(uint32_t, i, 0u, 512u) g16[i] = dp[i];
        g32 = (uint32_t*)(sst + off[SL_AP]);
        LANE_FOR(uint32_t, i, 0u, 16u) g32[i] = ap[i];
        if (!LIT_LDS) SPILL_FENCE();   // the coders' last HBM stores before they are copied
        g16 = (uint16_t*)(sst + off[SL_LIT]);
        LANE_FOR(uint32_t, i, 0u, nlit) g16[i] = lit[i];
    }
    // returns now_pos; every Encoder field a CodeOneBlock boundary carries, as saved
    FI uint32_t load_state() {
        uint32_t off[SL_COUNT];
        slice_layout(pb, lc, lp, tsize, off);
        const uint32_t nlit = 0x300u << (lc + lp);
        const uint16_t* g16 = (const uint16_t*)(sst + off[SL_PROBS]);
        LANE_FOR(uint32_t, i, 0u, (uint32_t)E_COUNT) probs[i] = g16[i];
        g16 = (const uint16_t*)(sst + off[SL_LENP]);
        LANE_FOR(uint32_t, i, 0u, (2u << pb) * tsize) lenp[i] = g16[i];
        const uint32_t* g32 = (const uint32_t*)(sst + off[SL_LENC]);
        LANE_FOR(uint32_t, i, 0u, 32u) lenc[i] = g32[i];
        g16 = (const uint16_t*)(sst + off[SL_PSP]);
        LANE_FOR(uint32_t, i, 0u, 256u) psp[i] = g16[i];
        g16 = (const uint16_t*)(sst + off[SL_DP]);
        LANE_FOR(uint32_t, i, 0u, 512u) dp[i] = g16[i];
        g32 = (const uint32_t*)(sst + off[SL_AP]);
        LANE_FOR(uint32_t, i, 0u, 16u) ap[i] = g32[i];
        g16 = (const uint16_t*)(sst + off[SL_LIT]);
        LANE_FOR(uint32_t, i, 0u, nlit) lit[i] = g16[i];
        if (!LIT_LDS) SPILL_FENCE();
        LANE_FENCE();
        LANE_FOR(uint32_t, i, 0u, (uint32_t)E_PSLOT) dmp[i] = price0(probs[i]) | (price1(probs[i]) << 16);
        LANE_FENCE();
        const uint32_t* sc = (const uint32_t*)(sst + off[SL_SCALARS]);
        const uint32_t now_pos = uni32(sc[SS_NOW_POS]);
        state = uni32(sc[SS_STATE]); prev_byte = uni32(sc[SS_PREV_BYTE]);
        rd0 = uni32(sc[SS_REP0]); rd1 = uni32(sc[SS_REP1]); rd2 = uni32(sc[SS_REP2]); rd3 = uni32(sc[SS_REP3]);
        match_price_count = uni32(sc[SS_MATCH_PRICE_COUNT]); align_price_count = uni32(sc[SS_ALIGN_PRICE_COUNT]);
        if (uni32(sc[SS_MAGIC]) != kSliceMagic || now_pos == 0 || now_pos >= n) bad = 10;
        mfpos = now_pos;
        return now_pos;
    }

    FI void run() {   // Encoder.Code: SetStreams + CodeOneBlock/encodeOne (Encoder.java:843-936, 1046-1077)
#ifdef LZG_PROF
        for (int k = 0; k < kProfSlots; k++) prof[k] = 0;
#endif
        const uint32_t nlit = 0x300u << (lc + lp);
        rp0 = rp1 = rp2 = rp3 = 0;
        rpos = 0; overflow = 0; bad = 0;
        longest_found = 0; opt_end = 0; opt_cur = 0; additional_offset = 0;
        longest_len = 0; num_pairs = 0; mfpos = 0;
        ring_base = 0x80000000u;   // force a fill at the first read (streams < 2 GiB)
        uint32_t now_pos = 0;
        bool resumed = false;
        if constexpr (kSliced) resumed = sresume != 0;
        if (resumed) {   // the sliced encode: a CodeOneBlock boundary of an earlier launch
            now_pos = load_state();
            if (bad) return;
        } else {
        LANE_FOR(uint32_t, i, 0u, (uint32_t)E_COUNT) probs[i] = kBitModelTotal >> 1;
        LANE_FOR(uint32_t, i, 0u, (uint32_t)E_PSLOT) dmp[i] = price0(kBitModelTotal >> 1) | (price1(kBitModelTotal >> 1) << 16);
        LANE_FOR(uint32_t, i, 0u, nlit) lit[i] = kBitModelTotal >> 1;
        LANE_FOR(uint32_t, i, 0u, 256u) psp[i] = 0;
        if (!LIT_LDS) SPILL_FENCE();
        LANE_FENCE();
        state = 0; prev_byte = 0;
        rd0 = rd1 = rd2 = rd3 = 0;
        match_price_count = 0; align_price_count = 0;
        DBG(1, 1);
        fill_distances_prices();
        DBG(1, 2);
        fill_align_prices();
        DBG(1, 3);
        for (uint32_t ps = 0; ps < (1u << pb); ps++) { update_len_table(0, ps); update_len_table(1, ps); }
        DBG(1, 4);
        }

        cold->prio.start(g_enc_sched, n, lane_id());
        if (!resumed) {
        if (avail() == 0) { flush(0); return; }
        read_match_distances();
        DBG(1, 5);
        encode_symbol(-1, 1, now_pos, byte_at(0 - additional_offset), 0, false);   // Encoder.java:860-878
        additional_offset--;
        now_pos++;
        if (avail() == 0) { flush(now_pos); return; }
        }
        DBG(1, 6);
        for (;;) {
            int32_t back;
            refresh_lane();
            DBG(2, now_pos);
            DBG(3, mfpos);
#ifdef LZG_PROF
            const uint64_t tg = PCLK();
#endif
            uint32_t sym_slot;
            uint32_t len = get_optimum(now_pos, &back, &sym_slot);
            PEND(PF_GETOPT, tg);
            DBG(4, len);
            if (bad || len == 0 || now_pos + len > n) { if (!bad) bad = 5; return; }
            PBEGIN(te);
            if (len == 1 && back == -1) {
                // literal: its byte, match byte and previous byte were recorded when the
                // position was parsed (o_bytes); a rep or match codes no byte
                // The match byte was taken with the rep0 of the slot's own best path; a
                // two-step candidate's middle literal can sit on a path with another rep0
                // (then the byte is re-read). Slot 0 always used the current rep0.
                const uint32_t top = opt_end > 0 ? (uint32_t)opt_end - 1 : 0u;   // behind fields written: slots <= top
                const bool fs_ = b_in(sym_slot, top);
                const uint32_t b = fs_ ? bytes_at<true>(sym_slot, top) : bytes_at(sym_slot, top);
                const uint32_t r0 = fs_ ? back_at<true>(sym_slot, 0, top) : back_at(sym_slot, 0, top);
                prev_byte = (b >> 16) & 0xFFu;
                uint32_t mb = (b >> 8) & 0xFFu;
                if (sym_slot != 0 && r0 != rd0) mb = byte_at((int32_t)(0 - rd0 - 1) - additional_offset);
                encode_symbol(-1, 1, now_pos, b & 0xFFu, mb, false);
            } else {
                encode_symbol(back, len, now_pos, 0, 0, false);
            }
            additional_offset -= (int32_t)len;
            now_pos += len;
            PEND(PF_ENCODE, te);
            if (additional_offset == 0) {
                PBEGIN(tt);
                if (match_price_count >= (1u << 7)) fill_distances_prices();
                if (align_price_count >= (uint32_t)kAlignTableSize) fill_align_prices();
                PEND(PF_TABLES, tt);
                cold->prio.update(now_pos, lane_id());
                if (avail() == 0) { flush(now_pos); return; }
                if constexpr (kSliced) {   // a slice ends at the first block boundary past its stop
                    if (now_pos >= sstop) { rec_store_tail(); save_state(now_pos, 0); return; }
                }
            }
        }
    }
};

// LDS layout of one stream's workgroup; shared by the kernel (carving) and
// the host (dynamic LDS size). Regions are 16-byte aligned.
enum { L_PP, L_PROBS, L_DMP, L_LENP, L_LENC, L_PSP, L_DP, L_AP, L_TP, L_MDBUF, L_RINFO, L_RPAIRS, L_OPRICE,
       L_OPP, L_OBP, L_OBP2, L_OBACKS, L_OBYTES, L_TPBUF, L_RBUF, L_COLD, L_LIT, L_COUNT };
__host__ __device__ constexpr uint32_t enc_lds_layout_p(uint32_t fb, uint32_t pb, uint32_t lc, uint32_t lp, uint32_t lit_in_lds,
                                                      uint32_t pair_bytes, uint32_t len_table_size, uint32_t* off) {
    const uint32_t md_cap = fb + 2;   // pairs per position <= fb (+1 clamp slot)
    const uint32_t sz[L_COUNT] = {
        512 * 2, prob_count(pb) * 2 + 2, dm_count(pb) * 4 + 4, 2 * (1u << pb) * len_table_size * 2, 2 * 16 * 4, 256 * 2, 512 * 2, 16 * 4,
        0u /* L_TP: unused (tempPrices are L_TPBUF) */, md_cap * pair_bytes, kRing * 4,
        kRing * kInlinePairs * pair_bytes,
        (kOptLds + 2) * 4, (kOptLds + 2) * 4, (kOptLds + 2) * 4, (kOptLds + 2) * 4, 4 * kOptLds * 4, kOptLds * 4, kTpBytes, kRbuf * 2 + 2, 128u /* Enc::Cold */,
        lit_in_lds ? (0x300u << (lc + lp)) * 2 + 2 : 0u};
    uint32_t o = 0;
    for (int i = 0; i < L_COUNT; i++) { if (off) off[i] = o; o += (sz[i] + 15) & ~15u; }
    return o;
}
__host__ __device__ inline uint32_t enc_lds_layout(const EncArgs& a, uint32_t* off) {
    return enc_lds_layout_p(a.fb, a.pb, a.lc, a.lp, a.lit_in_lds, a.pair_bytes, a.len_table_size, off);
}
// the bench parameters' layout (SPEC = 1: fb 32, lc 3, lp 0, pb 2), by pair width and literal-coder placement
template <int PAIR_BYTES, bool LIT>
constexpr uint32_t kSpec1LdsBytes = enc_lds_layout_p(32, 2, 3, 0, LIT ? 1u : 0u, PAIR_BYTES, 31, nullptr);

// SPEC = 1: the level-5 parameters of bench.py (fb 32, lc 3, lp 0, pb 2, no end
// marker) as compile-time constants; SPEC = 2: any parameters with fb <= 32;
// SPEC = 0: fb > 32. SPEC 1 and 2 keep _optimum in the LDS ring.
template <typename PairT, bool LIT_LDS, int PBS, int SPEC>
__global__ void __launch_bounds__(kWave, 4) enc_kernel(EncArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t* sm = smem;
    // SPEC 1: a static array, so every LDS offset folds into its ds instruction (other
    // kernels: a 16-byte placeholder, the dynamic array is theirs)
    __shared__ __attribute__((aligned(16))) uint8_t smem_s[SPEC == 1 ? kSpec1LdsBytes<(int)sizeof(PairT), LIT_LDS> : 16u];
    if constexpr (SPEC == 1) sm = smem_s;   // measured: one stream -9 %, 512 streams -10 %, 4096 flat (round 5)
    Enc<PairT, LIT_LDS, PBS, (SPEC != 0)> e;   // SPEC 1 and 2: fb <= 32, the _optimum ring
    e.lane_v = threadIdx.x % kWave;
    if (SPEC == 1) {
        e.fb = 32; e.lc = 3; e.lp = 0; e.pb = 2; e.ps_mask = 3; e.eos = 0; e.tsize = 31;
    } else {
        e.fb = a.fb; e.lc = a.lc; e.lp = a.lp; e.pb = a.pb; e.ps_mask = (1u << a.pb) - 1; e.eos = a.eos;
        e.tsize = a.len_table_size;
    }
    e.dist_table_size = a.dist_table_size;
    uint32_t off[L_COUNT];
    {
        EncArgs la = a;   // SPEC: the layout folds to constants (immediate LDS offsets, no SGPR per region)
        if (SPEC == 1) { la.fb = 32; la.pb = 2; la.lc = 3; la.lp = 0; la.lit_in_lds = LIT_LDS ? 1 : 0; la.pair_bytes = (uint32_t)sizeof(PairT); la.len_table_size = 31; }
        enc_lds_layout(la, off);
    }
    e.pp = (uint16_t*)(sm + off[L_PP]);
    e.probs = (uint16_t*)(sm + off[L_PROBS]);
    e.lenp = (uint16_t*)(sm + off[L_LENP]);
    e.lenc = (uint32_t*)(sm + off[L_LENC]);
    e.psp = (uint16_t*)(sm + off[L_PSP]);
    e.dp = (uint16_t*)(sm + off[L_DP]);
    e.ap = (uint32_t*)(sm + off[L_AP]);
    e.tp = (uint16_t*)(sm + off[L_TPBUF]);   // tempPrices (FillDistancesPrices' scratch), aliasing the window
    e.win = sm + off[L_TPBUF];
    e.dmp = (uint32_t*)(sm + off[L_DMP]);
    e.md_buf = (PairT*)(sm + off[L_MDBUF]);
    e.mdp = e.md_buf;
    e.ring_info = (uint32_t*)(sm + off[L_RINFO]);
    e.ring_pairs = (PairT*)(sm + off[L_RPAIRS]);
    e.o_price = (uint32_t*)(sm + off[L_OPRICE]);
    e.o_pp = (uint32_t*)(sm + off[L_OPP]);
    e.o_bp = (int32_t*)(sm + off[L_OBP]);
    e.o_bp2 = (int32_t*)(sm + off[L_OBP2]);
    e.o_backs = (uint32_t*)(sm + off[L_OBACKS]);
    e.o_bytes = (uint32_t*)(sm + off[L_OBYTES]);
    e.rbuf = (uint16_t*)(sm + off[L_RBUF]);
    e.cold = (typename Enc<PairT, LIT_LDS, PBS, (SPEC != 0)>::Cold*)(sm + off[L_COLD]);
    uint8_t* scratch = a.scratch + (size_t)blockIdx.x * a.scratch_stride;
    e.spill = __builtin_amdgcn_make_buffer_rsrc(scratch, 0, kNumOpts * 4 * 10, 0x00020000);
    uint16_t* lit_g = (uint16_t*)(a.lit_scratch + (size_t)blockIdx.x * a.lit_stride);
    if (LIT_LDS) e.lit = (uint16_t*)(sm + off[L_LIT]);
    else e.lit = lit_g;
    for (int i0 = 0; i0 < 512; i0 += kWave) e.pp[i0 + e.lane_v] = (uint16_t)c_tab.prices[i0 + e.lane_v];
    LANE_FENCE();
    e.dbg = a.dbg;
#ifdef LZG_DEBUG
    if (e.dbg && blockIdx.x == 0 && e.lane_v == 0) __hip_atomic_store(e.dbg, 7u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
    e.pairs = a.pairs;
    e.ovf_off = a.ovf_off;
    e.ovf = (const PairT*)a.ovf;
    // One workgroup per stream, longest first (order[]): the dispatcher is the
    // work queue, so the kernel has no outer loop and every wave retires at
    // the end of its stream.
    // wave-uniform by construction; readfirstlane keeps them (and the buffer
    // descriptor built from them) in SGPRs, so buffer loads need no waterfall loop
    const int s = __builtin_amdgcn_readfirstlane((int)a.order[blockIdx.x]);
    if (s < 0 || s >= a.nstreams) return;   // a corrupt order entry: touch nothing (the host checked the order it wrote)
    if (uni64(a.offs[s + 1]) < uni64(a.offs[s]) || uni64(a.rec_offs[s + 1]) < uni64(a.rec_offs[s])) {
        if (e.lane_v == 0) { a.rec_lens[s] = 0; a.out_lens[s] = 9ull << 32; a.status[s] = LZMA_E_INTERNAL; }
        return;
    }
    e.gbase = uni64(a.offs[s]);
    e.n = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uni64(a.offs[s + 1]) - e.gbase));
    e.in = a.in + e.gbase;
    e.inb = __builtin_amdgcn_make_buffer_rsrc((void*)e.in, 0, e.n, 0x00020000);
    if constexpr (kSliced) {   // the stream's own state region
        e.sst = a.slice_state + (size_t)s * a.slice_stride;
        e.sstop = a.slice_stop;
        e.sresume = a.slice_resume;
    }
    const uint64_t ro = uni64(a.rec_offs[s]);
    e.recs = a.recs + ro;
    e.rcap = uni64(a.rec_offs[s + 1]) - ro;
#ifdef LZG_DEBUG
    if (e.dbg && e.lane_v == 0) __hip_atomic_store(e.dbg + 8, (uint32_t)s + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#endif
#ifdef LZG_PROF
    const uint64_t t_run = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    e.run();
    e.cold->prio.finish(e.lane_v);
#ifdef LZG_PROF
    e.prof[PF_TOTAL] = __builtin_amdgcn_s_memtime() - t_run;
    e.prof[PF_T0] = rt0;   // 100 MHz wall clock: where each stream ran
    e.prof[PF_T1] = __builtin_amdgcn_s_memrealtime();
    // HW_REG_HW_ID (cu / sh / se / simd) and HW_REG_XCC_ID
    e.prof[PF_HWID] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4) | ((uint64_t)__builtin_amdgcn_s_getreg((15 << 11) | 20) << 32);
    if (e.lane_v == 0 && a.prof)
        for (int k = 0; k < kProfSlots; k++) a.prof[(size_t)s * kProfSlots + k] = e.prof[k];
#endif
    if (e.overflow && !e.bad) e.bad = 7;   // record region smaller than rc_record_bound(): a bug, not the data
    if (e.lane_v == 0) {
        a.rec_lens[s] = e.rpos;
        if (e.bad) a.out_lens[s] = ((uint64_t)e.bad << 32) | e.mfpos;
        a.status[s] = e.bad ? LZMA_E_INTERNAL : LZMA_OK;
    }
}

#if !LZG_ENC_SLICED   // shared by both parsers: defined once, in the plain one's translation unit
size_t enc_lds_bytes(const EncArgs& a) { return enc_lds_layout(a, nullptr); }

size_t enc_scratch_per_block(const Derived&) { return (size_t)kNumOpts * 4 * 10 + 256; }

size_t enc_lit_bytes(const Derived& d) { return ((size_t)0x300 << (d.lc + d.lp)) * 2 + 2; }   // + the sink entry

uint32_t enc_lit_in_lds(const Derived& d, int nstreams) {
    static const int force = exp_env("LZG_ENC_LITLDS") ? atoi(exp_env("LZG_ENC_LITLDS")) : -1;   // A/B runs
    const uint32_t bits = d.lc + d.lp;
    if (bits <= (uint32_t)kLitLdsMaxBits) return 1;
    if (force >= 0) return force != 0 && bits <= (uint32_t)kLitLdsMaxBitsFew;
    return nstreams <= kFewStreams && bits <= (uint32_t)kLitLdsMaxBitsFew;
}

int enc_grid(const Derived&, int nstreams) { return nstreams; }   // one workgroup per stream
#endif

template <typename PairT, bool LIT, int PBS, int SPEC>
static void launch_spec(Ctx* ctx, const EncArgs& a, int grid, size_t lds, hipStream_t st) {
    TimedLaunch tl(ctx, "enc_parse", st);
    if (SPEC == 1) lds = 0;   // the kernel's static array
    if (lds > 64 * 1024)
        hipFuncSetAttribute((const void*)enc_kernel<PairT, LIT, PBS, SPEC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((enc_kernel<PairT, LIT, PBS, SPEC>), dim3(grid), dim3(kWave), lds, st, a);
}

template <typename PairT, bool LIT, int PBS>
static void launch_one(Ctx* ctx, const EncArgs& a, int grid, size_t lds, hipStream_t st) {
    if constexpr (PBS == 2) {   // both pair widths: a single stream >= 8 MiB (config 4) takes the u64 form
        if (a.fb == 32 && a.lc == 3 && a.lp == 0 && a.pb == 2 && a.eos == 0) {
            launch_spec<PairT, LIT, PBS, 1>(ctx, a, grid, lds, st);
            return;
        }
    }
    if (a.fb <= 32) launch_spec<PairT, LIT, PBS, 2>(ctx, a, grid, lds, st);
    else launch_spec<PairT, LIT, PBS, 0>(ctx, a, grid, lds, st);
}

template <typename PairT, bool LIT>
static void launch_pb(Ctx* ctx, const EncArgs& a, int grid, size_t lds, hipStream_t st) {
    if (a.pb <= 2) launch_one<PairT, LIT, 2>(ctx, a, grid, lds, st);
    else launch_one<PairT, LIT, 4>(ctx, a, grid, lds, st);
}

int launch_encoder(Ctx* ctx, const EncArgs& a0, bool wide_pairs, int grid, hipStream_t st) {
    if (a0.pair_bytes != (wide_pairs ? 8u : 4u)) return ctx->fail(LZMA_E_INTERNAL, "pair width mismatch");
    EncArgs a = a0;
    size_t lds = enc_lds_bytes(a);
    // + the 16-byte static placeholder every kernel but SPEC 1 declares beside its dynamic LDS
    if (lds + 16 > 160 * 1024) return ctx->fail(LZMA_E_PARAM, "encoder LDS %zu too large", lds);
#ifdef LZG_ONLY_SPEC1_LIT   // code-inspection builds (assembly of one kernel family)
    if (!wide_pairs) {
        if (a.lit_in_lds) launch_spec<uint32_t, true, 2, 1>(ctx, a, grid, lds, st);
        else launch_spec<uint32_t, false, 2, 1>(ctx, a, grid, lds, st);
    }
#else
    if (wide_pairs) {
        if (a.lit_in_lds) launch_pb<uint64_t, true>(ctx, a, grid, lds, st);
        else launch_pb<uint64_t, false>(ctx, a, grid, lds, st);
    } else {
        if (a.lit_in_lds) launch_pb<uint32_t, true>(ctx, a, grid, lds, st);
        else launch_pb<uint32_t, false>(ctx, a, grid, lds, st);
    }
#endif
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "enc launch: %s", hipGetErrorString(e));
    return LZMA_OK;
}

#if LZG_ENC_SLICED
}  // namespace sliced

int launch_encoder_sliced(Ctx* ctx, const EncArgs& a, bool wide_pairs, int grid, hipStream_t st) {
    if (!a.slice_state) return ctx->fail(LZMA_E_INTERNAL, "sliced encode without a state region");
    return sliced::launch_encoder(ctx, a, wide_pairs, grid, st);
}
size_t enc_slice_state_bytes(const Derived& d) {
    return sliced::slice_layout(d.pb, d.lc, d.lp, d.len_table_size, nullptr);
}
#endif
}  // namespace lzg
