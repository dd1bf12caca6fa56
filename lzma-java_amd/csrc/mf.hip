// mf.hip -- phase 1 of the encoder: the BT2/BT4 binary-tree match finder of
// src/main/java/SevenZip/Compression/LZ/BinTree.java, computed for every
// position of a batch of independent streams at once.
//
// Why this is legal: the match list of position P depends
// only on (input, dict, fb, mf), never on parser decisions, because Skip and
// fillMatches make identical tree updates (BinTree.java:249-256 vs 335-339).
// A position's tree only ever links positions of the same hash4 bucket, so
// every bucket is an independent sequential simulation:
//   K1 mf_keys     hash every position (BinTree.java:170-178), key = (stream, hv)
//   K2 radix sort  (stream, hv) stable => each bucket a contiguous, position-
//                  ordered segment; hash2/hash3 "last occurrence" likewise
//   K3 mf_links    prev-in-bucket for hash2/hash3; bucket (chain) heads
//   K4 mf_walk     one lane per bucket: replays BinTree.fillMatches0
//                  (:152-273) for the bucket's positions in order, with the
//                  son[] links indexed by sorted bucket index (window expiry
//                  via matchMinPos makes cyclic reuse unobservable).
// Output per position: a record (lzma_common.h store_rec) of kInlinePairs
// packed pairs and info = count | main_len << 16 (main_len = longest pair
// extended past fb as Encoder.ReadMatchDistances does, Encoder.java:275-287);
// the pairs past kInlinePairs go to an overflow pool.
#include "lzma_common.h"
#include "runtime.h"

#include <cstdio>

namespace lzg {

static __constant__ Tables c_tab = make_tables();

constexpr uint64_t kSentinel = ~0ull;
constexpr uint32_t kSentinel32 = ~0u;

__device__ inline int find_stream(const uint64_t* offs, int nstreams, uint64_t g) {
    // largest s with offs[s] <= g (offs has nstreams+1 entries, offs[nstreams] = total)
    int lo = 0, hi = nstreams;  // answer in [lo, hi)
    while (hi - lo > 1) {
        int mid = (lo + hi) >> 1;
        if (offs[mid] <= g) lo = mid; else hi = mid;
    }
    return lo;
}

template <bool BT4>
__global__ void __launch_bounds__(256) mf_keys_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ offs,
                                                      int nstreams, uint64_t total, MfArgs a) {
    // one position per thread; the block's first position gives a wave-uniform
    // (scalar) stream search, and a lane past a stream end steps forward
    const uint64_t g0 = blockIdx.x * (uint64_t)blockDim.x;
    const uint64_t g = g0 + threadIdx.x;
    int s = find_stream(offs, nstreams, g0 < total ? g0 : total - 1);
    while (s + 1 < nstreams && offs[s + 1] <= g) s++;
    if (g < total) {
        uint64_t base = offs[s], n = offs[s + 1] - base, p = g - base;
        uint64_t rem = n - p;
        uint32_t len_limit = rem < a.fb ? (uint32_t)rem : a.fb;
        if (len_limit < a.min_match_check) {   // BinTree.java:153-162: no insertion
            a.k4[g] = kSentinel;
            if (BT4) { a.k3[g] = kSentinel32; a.k2[g] = kSentinel32; }
            // the walk skips this position: its record says "no pairs" (every other
            // position's record is written by the walk)
            a.mrec[g * a.rec_vecs + a.rec_vecs - 1] = v4u32{0u, 0u, 0u, 0u};
            return;
        }
        uint32_t b0 = in[g], b1 = in[g + 1];
        if (BT4) {
            uint32_t b2 = in[g + 2], b3 = in[g + 3];
            uint32_t temp = c_tab.crc[b0] ^ b1;
            uint32_t h2 = temp & 1023u;
            temp ^= b2 << 8;
            uint32_t h3 = temp & 0xFFFFu;
            uint32_t hv = (temp ^ (c_tab.crc[b3] << 5)) & a.hash_mask;
            a.k4[g] = ((uint64_t)s << a.hash_bits) | hv;
            a.k3[g] = ((uint32_t)s << 16) | h3;
            a.k2[g] = ((uint32_t)s << 10) | h2;
        } else {
            a.k4[g] = ((uint64_t)s << 16) | (b0 ^ (b1 << 8));
        }
    }
}

// prev-in-bucket for a position-ordered sorted key array (hash2 / hash3 heads).
// One item per thread, blocks mapped XCD-aware (XCD x takes the x-th eighth of
// the array in order): the blocks resident on an XCD then scatter into a
// fraction of one stream's prev[] range, so its L2 assembles whole lines
// instead of writing back partial ones from all over the batch.
__global__ void __launch_bounds__(256) mf_prev_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                      uint64_t total, uint32_t* __restrict__ prev) {
    const uint32_t per_xcd = gridDim.x / 8;   // the host pads the grid to a multiple of 8
    const uint64_t blk = (uint64_t)(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    const uint64_t i = blk * blockDim.x + threadIdx.x;
    if (i >= total) return;
    uint32_t k = keys[i];
    if (k == kSentinel32) return;
    prev[vals[i]] = (i > 0 && keys[i - 1] == k) ? vals[i - 1] : kNoPos;
}

// Unaligned 8-byte little-endian load from a buffer padded by >= 16 bytes.
__device__ inline uint64_t load8(const uint8_t* p) {
    uintptr_t a = (uintptr_t)p;
    const uint64_t* q = (const uint64_t*)(a & ~(uintptr_t)7);
    uint32_t sh = (uint32_t)(a & 7) * 8;
    uint64_t lo = q[0], hi = q[1];
    return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

// hash2 "last occurrence" (BinTree.java:183-193) without a sort: hash2 has only
// 1024 values, so one wave sweeps its stream in position order with the heads in
// LDS. Per round of 64 positions, one ballot per hash bit gives each lane the lanes
// with its hash (wave-level multi-split); the nearest of them below the lane is its
// predecessor, else the head, and the highest of them updates the head. Reads of
// k2 are coalesced (position order).
// The same sweep emits the walk's inputs of every position, in position order (coalesced),
// into the position's own match-list record (the walk reads it before it writes the record):
// the first 16 bytes of the suffix, the hash2 and hash3 "last occurrence" (prev3 comes from
// mf_prev_kernel, which runs first) and whether their first bytes equal the position's
// (BinTree.java:184-207). A member then costs the walk one load of its record instead of
// five scattered loads (prefix, two candidates, their bytes).
__global__ void __launch_bounds__(64) mf_prev2_kernel(const uint64_t* __restrict__ offs, const uint32_t* __restrict__ k2,
                                                      const uint8_t* __restrict__ in, const uint32_t* __restrict__ prev3,
                                                      v4u32* __restrict__ recs, uint32_t rec_vecs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];   // dynamic LDS (the CPU emulation shares it)
    uint32_t* head = (uint32_t*)smem;                                   // [1024] last position per hash2
    uint8_t* hbyte = smem + 1024 * 4;                                   // [1024] its first byte
    const uint32_t lane = threadIdx.x;
    for (uint32_t k = lane; k < 1024; k += 64) { head[k] = kNoPos; hbyte[k] = 0; }
    __syncthreads();
    const uint32_t s = blockIdx.x;
    const uint64_t lo = offs[s], n = offs[s + 1] - lo;
    // Software pipeline: a round's prefix and hash3 byte are loaded during the round
    // before it, its key and prev3 two rounds ahead (the byte load depends on them: prev3
    // is defined where the key is live); the hash2 candidate's byte comes from the
    // candidate's lane (same round) or from LDS (head).
    auto key2 = [&](uint64_t i) { return i < n ? k2[lo + i] : kSentinel32; };
    auto pos3 = [&](uint64_t i) { return i < n ? prev3[lo + i] : kNoPos; };
    auto byte3 = [&](uint32_t k, uint32_t p) { return k != kSentinel32 && p != kNoPos ? (uint32_t)in[p] : 0u; };
    uint32_t nkey = key2(lane), nnkey = key2(lane + 64);
    uint64_t nc0 = load8(in + lo + lane), nc1 = load8(in + lo + lane + 8);   // the batch copy is padded
    uint32_t np3 = pos3(lane), nnp3 = pos3(lane + 64);
    uint32_t nb3 = byte3(nkey, np3);
    for (uint64_t r0 = 0; r0 < n; r0 += 64) {
        const uint64_t i = r0 + lane;
        const uint32_t key = nkey, p3 = np3, b3 = nb3;
        const uint64_t c0 = nc0, c1 = nc1;
        if (r0 + 64 < n) {
            nc0 = load8(in + lo + i + 64); nc1 = load8(in + lo + i + 72);
            nb3 = byte3(nnkey, nnp3);
            nkey = nnkey; np3 = nnp3;
            nnkey = key2(i + 128); nnp3 = pos3(i + 128);
        }
        const bool live = key != kSentinel32;   // sentinel: no insertion, no prev (as mf_prev_kernel)
        const uint32_t d = key & 1023u;
        uint64_t peers = __ballot(live);
        for (int b = 0; b < 10; b++) {
            const bool on = (d >> b) & 1u;
            const uint64_t m = __ballot(on);
            peers &= on ? m : ~m;
        }
        const uint64_t below = peers & ((1ull << lane) - 1);   // lane < 64
        const uint64_t above = lane == 63 ? 0ull : (peers & ~((2ull << lane) - 1));
        const uint32_t cur0 = (uint32_t)(c0 & 0xFFu);
        const uint32_t src = below ? 63u - (uint32_t)__builtin_clzll(below) : lane;
        const uint32_t bsh = (uint32_t)__shfl((int)cur0, (int)src);   // every lane takes part
        const uint32_t hd = live ? head[d] : kNoPos;
        const uint32_t hb = live ? (uint32_t)hbyte[d] : 0u;
        __builtin_amdgcn_wave_barrier();
        if (live) {
            const uint32_t p2 = below ? (uint32_t)(lo + r0) + src : hd;
            const uint32_t b2 = below ? bsh : hb;
            if (above == 0) { head[d] = (uint32_t)(lo + i); hbyte[d] = (uint8_t)cur0; }
            const uint32_t f2 = p2 != kNoPos && b2 == cur0, f3 = p3 != kNoPos && b3 == cur0;
            v4u32* rp = recs + (lo + i) * rec_vecs;
            rp[0] = v4u32{(uint32_t)c0, (uint32_t)(c0 >> 32), (uint32_t)c1, (uint32_t)(c1 >> 32)};
            rp[1] = v4u32{p2, p3, f2 | (f3 << 1), 0u};
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// exclusive prefix sum of v over the block's threads; wsum: (blockDim / 64) words of LDS.
// One block barrier; the caller synchronises before wsum is written again (or passes
// another wsum): a wave that leaves the barrier early must not overwrite words the
// slower waves are still reading.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* wsum) {
    const uint32_t tid = threadIdx.x, lane = tid % 64, w = tid / 64;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, (unsigned)o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t q = 0; q < w; q++) before += wsum[q];
    return before + x - v;
}

// Long chains first, across all streams. A bucket's walk is serial, so a long
// one is the walk's tail: in stream order, the long buckets of the last streams
// start when their stream's turn comes and finish long after the short ones.
// Chains of kWalkLong or more members are therefore walked by the blocks at the
// front of the grid, longest length class (floor(log2 len)) first, beside the
// stream-ordered short ones (TEXT walk 929 -> 757 ms, BENCH 138 -> 132 ms). Order
// within a class is free: a chain's walk touches only its own positions, nodes
// and records. mf_chains_kernel lists them (unordered) and counts the classes.
constexpr uint32_t kWalkLong = 256;
constexpr uint32_t kWalkCapPct = 8;          // long chains' share of the positions (lower bound) that caps the walk
constexpr size_t kWalkCapLds = 40 * 1024;    // LDS per 64-lane block under the cap: 4 blocks per CU

// Walk-order key of a chain: longest first (lanes of one wave walk similar-length
// buckets); exact below 128, then 8 steps per doubling. Only the order depends on it.
__device__ __forceinline__ uint32_t chain_order_key(uint32_t len) {
    uint32_t f = len;
    if (len >= 128) {
        const uint32_t lg = 31u - (uint32_t)__clz((int)len);                 // >= 7
        f = 128u + 8u * (lg - 7u) + ((len >> (lg - 3u)) & 7u);
        if (f > 255u) f = 255u;
    }
    return 255u - f;
}

// The chain (bucket) lists of one stream, one workgroup per stream: chain k of the
// stream (its k-th bucket in sorted order) at index lo + k gets its first sorted index,
// its length and its walk-order key (the order sort takes index lo + k as the value);
// seg_end[s] = lo + chains.
// Sentinel keys (no insertion) sort last in their stream and form no chain.
constexpr uint32_t kChainThreads = 256, kChainItems = 4;
__global__ void __launch_bounds__(kChainThreads) mf_chains_kernel(const uint64_t* __restrict__ offs, const uint64_t* __restrict__ keys,
                                                                   uint32_t* __restrict__ chain_start, uint32_t* __restrict__ chain_len,
                                                                   uint32_t* __restrict__ okey,
                                                                   uint64_t* __restrict__ seg_end, uint32_t long_min,
                                                                   uint32_t* __restrict__ cls, uint32_t* __restrict__ long_raw) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];   // dynamic LDS (the CPU emulation shares it)
    uint32_t* wsum = (uint32_t*)smem;                                   // [kChainThreads / 64]: the head-count scan
    uint32_t* wsum2 = wsum + kChainThreads / 64;                        // [kChainThreads / 64]: the valid-item scan
    uint32_t* tile_tot = wsum2 + kChainThreads / 64;                    // [2]: heads, valid items
    const uint32_t tid = threadIdx.x, s = blockIdx.x;
    const uint64_t lo = offs[s], n = offs[s + 1] - lo;
    uint32_t run = 0, valid = 0;
    for (uint64_t t0 = 0; t0 < n; t0 += kChainThreads * kChainItems) {
        uint32_t head = 0, nv = 0;   // bit j: item j is a chain head
        const uint64_t b0 = t0 + (uint64_t)tid * kChainItems;
#pragma unroll
        for (uint32_t j = 0; j < kChainItems; j++) {
            const uint64_t i = b0 + j;
            if (i < n) {
                const uint64_t k = keys[lo + i];
                const bool live = k != kSentinel;
                nv += live;
                if (live && (i == 0 || keys[lo + i - 1] != k)) head |= 1u << j;
            }
        }
        const uint32_t cnt = (uint32_t)__builtin_popcount(head);
        const uint32_t ex = block_excl_scan(cnt, wsum);
        uint32_t c = run + ex;
#pragma unroll
        for (uint32_t j = 0; j < kChainItems; j++)
            if (head & (1u << j)) chain_start[lo + c++] = (uint32_t)(lo + b0 + j);
        if (tid == kChainThreads - 1) tile_tot[0] = ex + cnt;
        // a scan of its own words: with the same words, a wave through the first scan's barrier
        // overwrote them while slower waves still summed them (wrong chain starts; seen only when
        // other kernels share the CU and skew the waves: the encode-beside-decode fault of round 3)
        const uint32_t vex = block_excl_scan(nv, wsum2);   // barrier inside: tile_tot[0] is visible after it
        if (tid == kChainThreads - 1) tile_tot[1] = vex + nv;
        __syncthreads();
        run += tile_tot[0];
        valid += tile_tot[1];
        __syncthreads();
    }
    __syncthreads();
    const uint32_t nch = run;
    for (uint32_t c = tid; c < nch; c += kChainThreads) {
        const uint32_t st = chain_start[lo + c];
        const uint32_t en = c + 1 < nch ? chain_start[lo + c + 1] : (uint32_t)(lo + valid);
        const uint32_t len = en - st;
        chain_len[lo + c] = len;
        okey[lo + c] = chain_order_key(len);
        if (len >= long_min) {
            long_raw[atomicAdd(&cls[64], 1u)] = (uint32_t)(lo + c);
            atomicAdd(&cls[31 - __clz((int)len)], 1u);
        }
    }
    if (tid == 0) seg_end[s] = lo + nch;
}

// Exclusive scan of the streams' chain counts (one workgroup): chain_offs[s] = the
// stream's first index in the compacted walk order, chain_offs[nstreams] = all chains.
__global__ void __launch_bounds__(kChainThreads) mf_chain_scan_kernel(const uint64_t* __restrict__ offs, const uint64_t* __restrict__ seg_end,
                                                                       int nstreams, uint64_t* __restrict__ chain_offs) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t* wsum = (uint32_t*)smem;
    uint32_t* tile_tot = wsum + kChainThreads / 64;
    const uint32_t tid = threadIdx.x;
    uint64_t run = 0;
    for (int s0 = 0; s0 < nstreams; s0 += (int)kChainThreads) {
        const int s = s0 + (int)tid;
        const uint32_t v = s < nstreams ? (uint32_t)(seg_end[s] - offs[s]) : 0u;   // < 2^32 positions per pass
        const uint32_t ex = block_excl_scan(v, wsum);
        if (s < nstreams) chain_offs[s] = run + ex;
        if (tid == kChainThreads - 1) tile_tot[0] = ex + v;
        __syncthreads();
        run += tile_tot[0];
        __syncthreads();
    }
    if (tid == 0) chain_offs[nstreams] = run;
}


// First index r in [from, limit) with a[r] != b[r] (limit if none); when r < limit,
// *a_less = a[r] < b[r]. 16 bytes per iteration: both sides' words are loaded in
// one round trip, and the mismatching bytes come out of the loaded words (no
// separate byte loads for the tree-walk direction).
__device__ inline uint32_t cmp_run(const uint8_t* a, const uint8_t* b, uint32_t from, uint32_t limit, bool* a_less) {
    uint32_t len = from;
    while (len < limit) {
        const uint64_t a0 = load8(a + len), b0 = load8(b + len);
        const uint64_t a1 = load8(a + len + 8), b1 = load8(b + len + 8);
        uint64_t xa = a0, x = a0 ^ b0, xb = b0;
        uint32_t at = len;
        if (!x) { xa = a1; xb = b1; x = a1 ^ b1; at = len + 8; }
        if (x) {
            const uint32_t sh = (uint32_t)__builtin_ctzll(x) & ~7u;
            const uint32_t r = at + (sh >> 3);
            if (r >= limit) return limit;
            *a_less = ((xa >> sh) & 0xFFu) < ((xb >> sh) & 0xFFu);
            return r;
        }
        len += 16;
    }
    return limit;
}

// One binary-tree node of the walk, by sorted bucket index: the two links of
// BinTree._son (s0 = son[2i], s1 = son[2i + 1]; (1-based local position << 32) |
// (sorted index + 1), 0 = none) and the first 16 bytes of the member's suffix.
// A tree step loads one node (32 bytes, one request): its bytes for the compare
// and its links for the descent -- the walk reads the stream's bytes only for
// matches longer than 16.
struct alignas(32) WNode {
    uint64_t s0, s1, p0, p1;
};

// First index r in [from, min(16, limit)) where the 16-byte prefixes differ
// (cur = c0|c1, candidate = q0|q1); 16 if they agree through byte 15 (the
// caller continues in the stream); limit if r would reach it. *q_less = the
// candidate's byte < the current byte at r.
__device__ inline uint32_t pfx_cmp(uint64_t c0, uint64_t c1, uint64_t q0, uint64_t q1, uint32_t from, uint32_t limit,
                                   bool* q_less) {
    uint64_t xm, qa, ca;
    uint32_t at;
    if (from < 8) {
        xm = (c0 ^ q0) & (~0ull << (8 * from));
        qa = q0; ca = c0; at = 0;
        if (!xm) { xm = c1 ^ q1; qa = q1; ca = c1; at = 8; }
    } else {
        xm = (c1 ^ q1) & (~0ull << (8 * (from - 8)));
        qa = q1; ca = c1; at = 8;
    }
    if (!xm) return limit < 16 ? limit : 16;
    const uint32_t sh = (uint32_t)__builtin_ctzll(xm) & ~7u;
    const uint32_t r = at + (sh >> 3);
    if (r >= limit) return limit;
    *q_less = ((qa >> sh) & 0xFFu) < ((ca >> sh) & 0xFFu);
    return r;
}

// Common-prefix length of a[0..limit) and b[0..limit), starting at `from`.
__device__ inline uint32_t common_len(const uint8_t* a, const uint8_t* b, uint32_t from, uint32_t limit) {
    uint32_t len = from;
    while (len < limit) {
        uint64_t x = load8(a + len) ^ load8(b + len);
        if (x) {
            uint32_t r = len + (uint32_t)(__builtin_ctzll(x) >> 3);
            return r < limit ? r : limit;
        }
        len += 8;
    }
    return limit;
}

// scatter cursors of the long chains: the classes laid out longest first (one thread)
__global__ void mf_long_offsets_kernel(uint32_t* __restrict__ cls) {
    if (threadIdx.x != 0) return;
    uint32_t off = 0;
    for (int k = 31; k >= 0; k--) { cls[32 + k] = off; off += cls[k]; }
}
// the long chains in class order (longest class first)
__global__ void __launch_bounds__(256) mf_long_scatter_kernel(const uint32_t* __restrict__ long_raw, uint32_t n_long,
                                                              const uint32_t* __restrict__ chain_len, uint32_t* __restrict__ cls,
                                                              uint32_t* __restrict__ long_list) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_long) return;
    const uint32_t c = long_raw[i];
    long_list[atomicAdd(&cls[32 + 31 - __clz((int)chain_len[c])], 1u)] = c;
}

#ifdef LZG_WALK_WAVES   // experiment: a VGPR budget for more waves per SIMD (memory-level parallelism)
#define LZG_WALK_ATTR __attribute__((amdgpu_waves_per_eu(LZG_WALK_WAVES, LZG_WALK_WAVES)))
#elif defined(LZG_WALK_VGPRS)   // experiment: an explicit VGPR cap
#define LZG_WALK_ATTR __attribute__((amdgpu_num_vgpr(LZG_WALK_VGPRS)))
#else
#define LZG_WALK_ATTR
#endif
template <typename PairT, bool BT4>
__global__ void __launch_bounds__(64) LZG_WALK_ATTR mf_walk_kernel(const uint8_t* __restrict__ in, const uint64_t* __restrict__ offs,
                                                     const uint64_t* __restrict__ keys4, const uint32_t* __restrict__ vals4,
                                                     const uint32_t* __restrict__ chain_order,
                                                     const uint32_t* __restrict__ chain_start,
                                                     const uint32_t* __restrict__ chain_len,
                                                     uint64_t nchains,
                                                     const uint32_t* __restrict__ long_list, uint64_t n_long,
                                                     uint32_t long_blocks, uint32_t min_len,
                                                     MfArgs a, WNode* __restrict__ nodes, v4u32* __restrict__ recs,
                                                     uint32_t* __restrict__ ovf_off, PairT* __restrict__ ovf,
                                                     unsigned long long* __restrict__ ovf_used, uint64_t ovf_cap,
                                                     uint32_t ovf_stride,
                                                     int* __restrict__ err) {
    using PP = PairPack<PairT>;
    uint32_t c;
    // The walk trusts nothing it did not compute itself: a chain index, a chain's
    // extent, its stream and every member's position are range-checked, and a bad
    // one ends the lane with err = 4 (LZMA_E_INTERNAL on the host) instead of a
    // fault or a member loop that never ends.
    if (blockIdx.x < long_blocks) {   // the long chains, longest first, dealt over the XCDs in dispatch order
        const uint64_t li = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
        if (li >= n_long) return;
        c = long_list[li];
        if ((uint64_t)c >= a.total) { *err = 4; return; }
    } else {
        // XCD-aware mapping: the dispatcher places block b on XCD b % 8, so XCD x takes
        // the x-th eighth of the (stream-ordered) chain list and its L2 serves a few
        // streams (long_blocks and the grid are multiples of 8: b keeps its XCD)
        const uint32_t b = blockIdx.x - long_blocks;
        const uint32_t per_xcd = (gridDim.x - long_blocks) / 8;
        const uint64_t blk = (uint64_t)(b % 8) * per_xcd + b / 8;
        const uint64_t ci = blk * blockDim.x + threadIdx.x;
        if (ci >= nchains) return;
        c = chain_order[ci];
        if ((uint64_t)c >= a.total) { *err = 4; return; }
        if (chain_len[c] >= min_len) return;   // walked by the front blocks
    }
    uint64_t start = chain_start[c], end = start + chain_len[c];
    if (start == end) return;   // a stream's sentinel run
    if (end > a.total || end < start) { *err = 4; return; }
    if (end - start < a.walk_lo || end - start > a.walk_hi) return;   // timing experiment only (LZG_WALK_ONLY)
    uint64_t key = keys4[start];
    int s = (int)(key >> (BT4 ? a.hash_bits : 16));
    if (key == kSentinel || s < 0 || s >= a.nstreams) { *err = 4; return; }
    uint64_t base = offs[s], n = offs[s + 1] - base;
    const uint8_t* sb = in + base;          // stream bytes, 0-based
    const uint32_t fb = a.fb, cut = a.cut_value;
    const uint64_t cyc = a.cyc_size;
    uint32_t prev_local = 0;                // 1-based local position of previous bucket member, 0 = none
    // The tree nodes are indexed by the member's index in the sorted key array (not
    // by position): a bucket's tree lives in one contiguous run of WNodes, so a
    // walk touches a few cache lines instead of one random line per step.
    // Memory ordering matters here: on CDNA a load's wait also waits for every
    // store issued before it, so each step issues the next node's load before
    // its own link store, the pairs of a position stay in registers until the
    // position ends, and the newest member's node (the next position's first
    // tree node) is carried in registers instead of being re-read.
    WNode head{};                            // node of the previous member (valid when prev_local != 0)
    // Software pipeline over the bucket's members: the inputs of member i + 1 (its
    // prefix, its hash2/hash3 candidates' first bytes) and the candidates of member
    // i + 2 are loaded at the start of member i, so they arrive while member i walks
    // the tree instead of in front of member i + 1's walk.
    // BT4: a member's inputs (prefix, hash2 / hash3 candidates and whether their first
    // bytes match) are one 32-byte load of its record, written in position order by
    // mf_prev2_kernel; BT2 has no candidates and loads its prefix from the stream
    const uint32_t rv = a.rec_vecs;
    auto member_in = [&](uint64_t gi, uint64_t& c0_, uint64_t& c1_, uint32_t& v2_, uint32_t& v3_, uint32_t& f_) {
        if (BT4) {
            const v4u32* rp = recs + gi * rv;
            const v4u32 x0 = __builtin_nontemporal_load(rp), x1 = __builtin_nontemporal_load(rp + 1);
            c0_ = (uint64_t)x0[0] | ((uint64_t)x0[1] << 32); c1_ = (uint64_t)x0[2] | ((uint64_t)x0[3] << 32);
            v2_ = x1[0]; v3_ = x1[1]; f_ = x1[2];
        } else {
            c0_ = load8(sb + (gi - base)); c1_ = load8(sb + (gi - base) + 8);
            v2_ = v3_ = kNoPos; f_ = 0;
        }
    };
    uint64_t g = vals4[start];
    uint64_t g1 = start + 1 < end ? vals4[start + 1] : 0, g2 = start + 2 < end ? vals4[start + 2] : 0;
    uint64_t c0, c1;
    uint32_t pv2, pv3, fl;
    member_in(g, c0, c1, pv2, pv3, fl);
    for (uint64_t i = start; i < end; i++) {
        if (g - base >= n) { *err = 4; return; }   // a member outside its chain's stream
        const uint64_t g3 = i + 3 < end ? vals4[i + 3] : 0;
        uint64_t c0n = 0, c1n = 0;
        uint32_t pv2n = kNoPos, pv3n = kNoPos, fln = 0;
        if (i + 1 < end) member_in(g1, c0n, c1n, pv2n, pv3n, fln);   // arrives while member i walks
        uint32_t p = (uint32_t)(g - base);
        uint32_t pos = p + 1;               // BinTree 1-based position
        uint64_t rem = n - p;
        uint32_t len_limit = rem < fb ? (uint32_t)rem : fb;
        uint32_t match_min = (uint64_t)pos > cyc ? (uint32_t)(pos - cyc) : 0;
        const uint8_t* cur = sb + p;
        uint32_t cur_match = prev_local;
        uint32_t max_len = 1, cnt = 0;
        PairT q0 = 0, q1 = 0, q2 = 0, q3 = 0;   // the inline pairs, stored when the position ends
        PairT* ov = nullptr;
        bool ov_ok = false;
        // the last emitted pair stays in registers: the fb extension below must not
        // re-read it from memory (a failed overflow allocation leaves no copy there)
        uint32_t last_l = 0, last_d = 0;
        auto emit = [&](uint32_t l, uint32_t d) {
            const PairT v = PP::pack(l, d);
            if (cnt < kInlinePairs) {
                q0 = cnt == 0 ? v : q0; q1 = cnt == 1 ? v : q1; q2 = cnt == 2 ? v : q2; q3 = cnt == 3 ? v : q3;
            } else {
                if (ov == nullptr) {
                    // the pool is handed out in slots of ovf_stride pairs: a position
                    // takes at most one slot, so a 32-bit slot index always suffices
                    unsigned long long o = atomicAdd(ovf_used, 1ull);
                    ov_ok = (o + 1) * ovf_stride <= ovf_cap;
                    if (!ov_ok) { *err = 1; o = 0; }
                    ovf_off[g] = (uint32_t)o;
                    ov = ovf + o * ovf_stride;
                }
                if (ov_ok) ov[cnt - kInlinePairs] = v;
            }
            last_l = l;
            last_d = d;
            cnt++;
        };
        if (BT4) {   // hash2 / hash3 candidates, BinTree.java:183-207 (the byte checks: mf_prev2_kernel)
            uint32_t cm2 = pv2 == kNoPos ? 0 : (uint32_t)(pv2 - base) + 1;
            uint32_t cm3 = pv3 == kNoPos ? 0 : (uint32_t)(pv3 - base) + 1;
            if (cm2 > match_min && (fl & 1u)) { max_len = 2; emit(2, pos - cm2 - 1); }
            const uint32_t d2 = pos - cm2 - 1;   // the len-2 pair's distance, if it was emitted
            if (cm3 > match_min && (fl & 2u)) {
                if (cm3 == cm2) cnt--;
                max_len = 3;
                emit(3, pos - cm3 - 1);
                cm2 = cm3;
            }
            if (cnt != 0 && cm2 == cur_match) {
                cnt--;
                max_len = 1;
                if (cnt == 1) { last_l = 2; last_d = d2; }   // the len-2 pair is the last one again
            }
        }
        // this member's node: its links are set by its own walk (tracked in registers
        // while ptr0/ptr1 still point at it), its prefix is c0|c1
        WNode self{0, 0, c0, c1};
        bool p0_self = true, p1_self = true;   // ptr0 = son[2i + 1] (s1), ptr1 = son[2i] (s0)
        uint64_t* ptr0 = &nodes[i].s1;
        uint64_t* ptr1 = &nodes[i].s0;
        // the chain's last member: no later member walks the tree, so its links and its own
        // node are never read -- its walk stores only the match list
        const bool live_tree = i + 1 < end;
        auto put0 = [&](uint64_t v) { if (p0_self) self.s1 = v; else if (live_tree) *ptr0 = v; };
        auto put1 = [&](uint64_t v) { if (p1_self) self.s0 = v; else if (live_tree) *ptr1 = v; };
        uint64_t cur_idx = i - 1;           // sorted index of the head (valid while cur_match != 0)
        uint32_t len0 = a.direct_bytes, len1 = a.direct_bytes;
        if (!BT4 && cur_match > match_min) {   // BT2 direct byte check, BinTree.java:218-226
            if (sb[cur_match - 1 + 2] != cur[2]) { max_len = 2; emit(2, pos - cur_match - 1); }
        }
        WNode nd = head;                    // the first node visited is the previous member
        uint32_t count = cut;
        // direction of the previous step (0 none, 1 ptr0 side, 2 ptr1 side): a step that
        // goes the same way stores into the very slot it was reached through, which
        // already holds this node -- the store is skipped (no write, no vmcnt entry)
        uint32_t prev_dir = 0;
        for (;;) {   // BinTree.java:230-270
            if (cur_match <= match_min || count-- == 0) {
                // reached through a null link (nxt == 0): that slot already holds 0
                const bool null_in = cur_match == 0 && prev_dir != 0;
                if (!(null_in && prev_dir == 1)) put0(0);
                if (!(null_in && prev_dir == 2)) put1(0);
                break;
            }
            uint32_t delta = pos - cur_match;
            uint32_t len = len0 < len1 ? len0 : len1;
            // BinTree.java:243-248: the bytes equal at len => extend; the direction
            // (:259) compares the bytes at the first mismatch
            bool pby_less = false;
            uint32_t l2 = len < 16 ? pfx_cmp(c0, c1, nd.p0, nd.p1, len, len_limit, &pby_less) : len;
            if (l2 >= 16 && l2 < len_limit) l2 = cmp_run(sb + (cur_match - 1), cur, l2, len_limit, &pby_less);
            bool emit_now = false;
            if (l2 > len) {
                len = l2;
                if (max_len < len) {
                    max_len = len;
                    if (len == len_limit) { emit(len, delta - 1); put1(nd.s0); put0(nd.s1); break; }
                    emit_now = true;
                }
            }
            const uint64_t node = ((uint64_t)cur_match << 32) | (uint32_t)(cur_idx + 1);
            uint64_t nxt = pby_less ? nd.s1 : nd.s0;
            uint64_t* const here = pby_less ? &nodes[cur_idx].s1 : &nodes[cur_idx].s0;
            // a link always names an earlier member of this bucket: anything else is a
            // consistency failure, reported instead of followed
            if (nxt != 0 && ((uint64_t)(uint32_t)nxt - 1 < start || (uint64_t)(uint32_t)nxt - 1 >= i)) { *err = 3; nxt = 0; }
            if (nxt != 0) nd = nodes[(uint32_t)nxt - 1];   // issued before this step's stores
            if (pby_less) { if (prev_dir != 2) put1(node); ptr1 = here; p1_self = false; len1 = len; prev_dir = 2; }
            else { if (prev_dir != 1) put0(node); ptr0 = here; p0_self = false; len0 = len; prev_dir = 1; }
            if (emit_now) emit(len, delta - 1);
            if (nxt == 0) cur_match = 0;
            else { cur_idx = (uint32_t)nxt - 1; cur_match = (uint32_t)(nxt >> 32); }
        }
        uint32_t ml = 0;
        if (cnt > 0) {   // Encoder.ReadMatchDistances extension, Encoder.java:279-284
            ml = last_l;
            if (ml == fb) {
                uint32_t d1 = last_d + 1;
                uint64_t from = (uint64_t)p + ml;
                uint64_t lim = kMatchMaxLen - ml;
                if (from + lim > n) lim = n - from;
                ml += common_len(sb + from - d1, sb + from, 0, (uint32_t)lim);
            }
        }
        if (live_tree) nodes[i] = self;
        head = self;
        // outputs are touched once: non-temporal, so the stream's nodes and bytes keep the L2
        store_rec<PairT>(recs + g * rec_vecs<PairT>(), q0, q1, q2, q3, cnt | (ml << 16));
        prev_local = pos;
        g = g1; g1 = g2; g2 = g3;
        c0 = c0n; c1 = c1n;
        pv2 = pv2n; pv3 = pv3n; fl = fln;
    }
}

// ----------------------------------------------------------------- host side

static inline uint32_t bits_for(uint64_t v) { uint32_t b = 0; while (b < 64 && (v >> b) != 0) b++; return b; }

static inline unsigned grid_for(uint64_t n, unsigned block, unsigned cap = 65536) {
    uint64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    return (unsigned)(g < cap ? g : cap);
}

static MfArgs mf_args(const Derived& d, const MfBuffers& w, uint64_t total, int nstreams, bool wide_pairs) {
    MfArgs a{};
    a.fb = d.fb; a.min_match_check = d.min_match_check; a.hash_mask = d.hash_mask; a.hash_bits = d.hash_bits;
    a.cut_value = d.cut_value; a.cyc_size = d.cyc_size; a.direct_bytes = d.direct_bytes;
    a.walk_lo = 0; a.walk_hi = 0xFFFFFFFFu;
    a.total = total; a.nstreams = nstreams;
    if (const char* e = exp_env("LZG_WALK_ONLY")) {   // "lo,hi": a timing experiment; the output is incomplete
        unsigned lo = 0, hi = 0xFFFFFFFFu;
        if (sscanf(e, "%u,%u", &lo, &hi) >= 1) { a.walk_lo = lo; a.walk_hi = hi; }
    }
    a.k4 = w.k4; a.k3 = w.k3; a.k2 = w.k2; a.mrec = w.pairs; a.rec_vecs = wide_pairs ? rec_vecs<uint64_t>() : rec_vecs<uint32_t>(); a.prev3 = w.prev3;
    return a;
}

// K1..K4 for one batch, in two calls. in: padded device copy of the batch; offs: device
// stream offsets (nstreams+1). mf_front enqueues the keys, sorts and chain lists and
// returns; mf_back reads the chain count back (one host round trip), runs the walk and
// reads its verdict back. Fills w.pairs (records) / w.ovf_off / w.ovf.
// The long chains' scratch list: k4, dead since the hash4 sort (mf_chains_kernel fills it)
static uint32_t mf_long_min() {
    // LZG_WALK_LONG overrides the long-chain threshold (experiments; 4294967295 = stream order only)
    static const uint32_t long_min = exp_env("LZG_WALK_LONG") ? (uint32_t)strtoul(exp_env("LZG_WALK_LONG"), nullptr, 10) : kWalkLong;
    return long_min;
}

int mf_front(Ctx* ctx, const Derived& d, const uint8_t* in, const uint64_t* d_offs, int nstreams, uint64_t total,
             bool wide_pairs, MfBuffers& w, hipStream_t st) {
    if (total == 0) return LZMA_OK;
    if (total >= 0xFFFFFFFFull) return ctx->fail(LZMA_E_PARAM, "batch too large for 32-bit positions");
    MfArgs a = mf_args(d, w, total, nstreams, wide_pairs);
    const bool bt4 = d.hash_array != 0;
    const unsigned B = 256;
    {
        TimedLaunch tl(ctx, "mf_keys", st);
        const unsigned kgrid = (unsigned)((total + B - 1) / B);   // total < 2^32: fits
        if (bt4) hipLaunchKernelGGL((mf_keys_kernel<true>), dim3(kgrid), dim3(B), 0, st, in, d_offs, nstreams, total, a);
        else hipLaunchKernelGGL((mf_keys_kernel<false>), dim3(kgrid), dim3(B), 0, st, in, d_offs, nstreams, total, a);
    }
    LZG_TRACE(ctx, st, "mf_keys done (%llu positions)", (unsigned long long)total);
    int rc;
    if (bt4) {
        const unsigned prev_grid = (unsigned)(((total + B - 1) / B + 7) & ~7ull);   // total < 2^32: fits
        {
            TimedLaunch tl(ctx, "mf_sort", st);
            if ((rc = seg_radix_sort(ctx, false, w.k3, nullptr, w.ks, w.vs, w.son, w.son + total, w.hist, total, d_offs, nstreams, 16, st))) return rc;
        }
        hipLaunchKernelGGL(mf_prev_kernel, dim3(prev_grid), dim3(B), 0, st, (const uint32_t*)w.ks, w.vs, total, w.prev3);
        {   // after mf_prev: the walk-input records carry both candidates
            TimedLaunch tl(ctx, "mf_prev2", st);
            hipLaunchKernelGGL(mf_prev2_kernel, dim3(nstreams), dim3(64), 1024 * 5, st, d_offs, (const uint32_t*)w.k2, in,
                               (const uint32_t*)w.prev3, w.pairs, a.rec_vecs);
        }
    }
    {
        TimedLaunch tl(ctx, "mf_sort", st);
        if ((rc = seg_radix_sort(ctx, true, w.k4, nullptr, w.ks, w.vs, w.son, w.son + total, w.hist, total, d_offs, nstreams,
                                 (int)(bt4 ? d.hash_bits : 16), st))) return rc;
    }
    // chain lists and walk order: stream by stream (cache locality), longest chains first
    // within a stream (lanes of one wave walk similar-length buckets). The k2/k3 key
    // arrays are dead here and hold the order keys.
    uint32_t* okey = w.k2;
    uint32_t* okey_sorted = w.k3;
    uint32_t* long_raw = (uint32_t*)w.k4;   // dead since the hash4 sort
    const uint32_t long_min = mf_long_min();
    {
        TimedLaunch tl(ctx, "mf_sort", st);
        hipMemsetAsync(w.cls, 0, 96 * sizeof(uint32_t), st);
        hipLaunchKernelGGL(mf_chains_kernel, dim3(nstreams), dim3(kChainThreads), (2 * (kChainThreads / 64) + 2) * 4, st, d_offs, w.ks,
                           w.chain_start, w.chain_len, okey, w.seg_end, long_min, w.cls, long_raw);
        hipLaunchKernelGGL(mf_chain_scan_kernel, dim3(1), dim3(kChainThreads), (kChainThreads / 64 + 2) * 4, st, d_offs, w.seg_end,
                           nstreams, w.chain_offs);
        if ((rc = seg_radix_sort(ctx, false, okey, nullptr, okey_sorted, w.chain_order, w.son, w.son + total, w.hist, total,
                                 d_offs, nstreams, 8, st, w.seg_end, w.chain_offs))) return rc;
    }
    return LZMA_OK;
}

// pinned words of a slot: [0] chain count, [1] long-chain count, [2] the walk's verdict
// pinned words of a slot: [0] chain count, [1] long-chain count, [2] the walk's verdict,
// [4, 20): the long chains per length class (32 u32, mf_chains_kernel's cls[0..31])
constexpr int kPinSlotWords = 20;
static uint64_t* pin_slot(Ctx* ctx, int slot) { return ctx->pin_mf.as<uint64_t>() + kPinSlotWords * slot; }

int mf_count_enqueue(Ctx* ctx, const MfBuffers& w, int nstreams, hipStream_t st, int slot) {
    if (!ctx->pin_mf.ensure(2 * kPinSlotWords * sizeof(uint64_t))) return ctx->fail(LZMA_E_NOMEM, "pinned staging");
    if (!ctx->cnt_done[slot] && hipEventCreateWithFlags(&ctx->cnt_done[slot], hipEventDisableTiming) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "chain-count event");
    uint64_t* p_cnt = pin_slot(ctx, slot);
    p_cnt[0] = p_cnt[1] = 0;
    for (int k = 4; k < kPinSlotWords; k++) p_cnt[k] = 0;
    p_cnt[2] = 0;   // the walk's verdict (no walk: none)
    // sizes the walk grid: one host round trip per pass (pinned: see HostBuf)
    if (w.chain_offs &&
        (hipMemcpyAsync(p_cnt, w.chain_offs + nstreams, 8, hipMemcpyDeviceToHost, st) != hipSuccess ||
         hipMemcpyAsync(p_cnt + 1, w.cls + 64, 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
         hipMemcpyAsync(p_cnt + 4, w.cls, 32 * sizeof(uint32_t), hipMemcpyDeviceToHost, st) != hipSuccess))
        return ctx->fail(LZMA_E_DEVICE, "mf: chain count: %s", hipGetErrorString(hipGetLastError()));
    if (hipEventRecord(ctx->cnt_done[slot], st) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "mf: chain count: %s", hipGetErrorString(hipGetLastError()));
    return LZMA_OK;
}

int mf_walk_launch(Ctx* ctx, const Derived& d, const uint8_t* in, const uint64_t* d_offs, int nstreams, uint64_t total,
                   bool wide_pairs, MfBuffers& w, hipStream_t st, int slot) {
    if (hipEventSynchronize(ctx->cnt_done[slot]) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "mf: chain count: %s", hipGetErrorString(hipGetLastError()));
    if (total == 0) return LZMA_OK;
    MfArgs a = mf_args(d, w, total, nstreams, wide_pairs);
    const bool bt4 = d.hash_array != 0;
    const unsigned B = 256;
    uint32_t* long_raw = (uint32_t*)w.k4;            // k4 is dead since the hash4 sort: the long chains
    uint32_t* long_list = (uint32_t*)w.k4 + total;   // unordered, then in class order
    const uint32_t long_min = mf_long_min();
    uint64_t* p_cnt = pin_slot(ctx, slot);
    const uint64_t nchains = p_cnt[0];
    const uint32_t n_long = (uint32_t)p_cnt[1];   // the long chains (walked first)
    LZG_TRACE(ctx, st, "mf sorts + chain lists done");
    if (nchains > total || n_long > nchains)   // the grid below is sized from these: never launch on a bad count
        return ctx->fail(LZMA_E_INTERNAL, "mf: chain counts %llu / %u out of range", (unsigned long long)nchains, n_long);
    if (nchains == 0) return LZMA_OK;
    if (n_long) {
        TimedLaunch tl(ctx, "mf_sort", st);
        hipLaunchKernelGGL(mf_long_offsets_kernel, dim3(1), dim3(64), 0, st, w.cls);
        hipLaunchKernelGGL(mf_long_scatter_kernel, dim3((n_long + B - 1) / B), dim3(B), 0, st, long_raw, n_long, w.chain_len, w.cls,
                           long_list);
    }
    hipMemsetAsync(w.ovf_used, 0, sizeof(unsigned long long), st);
    hipMemsetAsync(w.err, 0, sizeof(int), st);
    {
        TimedLaunch tl(ctx, "mf_walk", st);
        const unsigned WB = 64;
        const unsigned long_blocks = (unsigned)(((n_long + WB - 1) / WB + 7) & ~7ull);
        unsigned grid = (unsigned)((nchains + WB - 1) / WB);
        grid = ((grid + 7) & ~7u) + long_blocks;   // multiples of 8 (XCD-aware mapping in mf_walk_kernel)
        // Waves per CU capped through dynamic LDS when long chains hold many of the positions:
        // a long chain's tree steps read 32-byte nodes all over its bucket's run, and with every
        // wave of the launch resident those reads thrash the XCD's L2; one walk wave per SIMD
        // lets them hit. TEXT (26 % of the positions in chains of 256 or more): walk 763 -> 696 ms;
        // BENCH (1.6 %) keeps every wave (a cap of 8 per CU cost it 10 %)
        // (profiles/r06/walk_split_text_caps.txt, ab/walk_cap_*.jsonl). LZG_WALK_LDS overrides (experiments).
        uint64_t long_members = 0;   // a lower bound: 2^class per chain
        const uint32_t* lcls = (const uint32_t*)(p_cnt + 4);
        for (int k = 0; k < 32; k++) long_members += (uint64_t)lcls[k] << k;
        const size_t walk_lds = exp_env("LZG_WALK_LDS") ? (size_t)atoi(exp_env("LZG_WALK_LDS"))
                                : (long_members * 100 >= total * (uint64_t)kWalkCapPct ? kWalkCapLds : 0);
        if (wide_pairs) {
            if (bt4) hipLaunchKernelGGL((mf_walk_kernel<uint64_t, true>), dim3(grid), dim3(WB), walk_lds, st, in, d_offs, w.ks, w.vs, w.chain_order, w.chain_start, w.chain_len, nchains, long_list, (uint64_t)n_long, long_blocks, long_min, a, (WNode*)w.son, w.pairs, w.ovf_off, (uint64_t*)w.ovf, w.ovf_used, w.ovf_cap, ovf_stride(d.fb), w.err);
            else hipLaunchKernelGGL((mf_walk_kernel<uint64_t, false>), dim3(grid), dim3(WB), walk_lds, st, in, d_offs, w.ks, w.vs, w.chain_order, w.chain_start, w.chain_len, nchains, long_list, (uint64_t)n_long, long_blocks, long_min, a, (WNode*)w.son, w.pairs, w.ovf_off, (uint64_t*)w.ovf, w.ovf_used, w.ovf_cap, ovf_stride(d.fb), w.err);
        } else {
            if (bt4) hipLaunchKernelGGL((mf_walk_kernel<uint32_t, true>), dim3(grid), dim3(WB), walk_lds, st, in, d_offs, w.ks, w.vs, w.chain_order, w.chain_start, w.chain_len, nchains, long_list, (uint64_t)n_long, long_blocks, long_min, a, (WNode*)w.son, w.pairs, w.ovf_off, (uint32_t*)w.ovf, w.ovf_used, w.ovf_cap, ovf_stride(d.fb), w.err);
            else hipLaunchKernelGGL((mf_walk_kernel<uint32_t, false>), dim3(grid), dim3(WB), walk_lds, st, in, d_offs, w.ks, w.vs, w.chain_order, w.chain_start, w.chain_len, nchains, long_list, (uint64_t)n_long, long_blocks, long_min, a, (WNode*)w.son, w.pairs, w.ovf_off, (uint32_t*)w.ovf, w.ovf_used, w.ovf_cap, ovf_stride(d.fb), w.err);
        }
    }
    LZG_TRACE(ctx, st, "mf_walk done (%llu chains)", (unsigned long long)nchains);
    if (hipMemcpyAsync(p_cnt + 2, w.err, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess)
        return ctx->fail(LZMA_E_DEVICE, "mf_walk: %s", hipGetErrorString(hipGetLastError()));
    return LZMA_OK;
}

// the walk's verdict, once the stream that launched it has passed its verdict copy
int mf_walk_result(Ctx* ctx, int slot) {
    const int32_t e = (int32_t)pin_slot(ctx, slot)[2];
    if (e == 3) return ctx->fail(LZMA_E_INTERNAL, "mf_walk: a tree link outside its bucket");
    if (e == 4) return ctx->fail(LZMA_E_INTERNAL, "mf_walk: a chain list entry out of range (index, extent, stream or member)");
    if (e) return LZMA_E_OVERFLOW;   // caller grows the overflow pool and retries
    return LZMA_OK;
}

int mf_back(Ctx* ctx, const Derived& d, const uint8_t* in, const uint64_t* d_offs, int nstreams, uint64_t total,
            bool wide_pairs, MfBuffers& w, hipStream_t st) {
    int rc;
    if ((rc = mf_count_enqueue(ctx, w, nstreams, st, 0)) || (rc = mf_walk_launch(ctx, d, in, d_offs, nstreams, total, wide_pairs, w, st, 0)))
        return rc;
    if (hipStreamSynchronize(st) != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "mf_walk: %s", hipGetErrorString(hipGetLastError()));
    return mf_walk_result(ctx, 0);
}

}  // namespace lzg
