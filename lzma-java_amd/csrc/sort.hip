// sort.hip -- the match finder's bucket sorts (mf.hip K2): a stable LSD radix
// sort of every stream's positions by the hash bits of their keys, one
// workgroup per stream.
//
// The positions of a pass are stream-major already (the walk and the hash2 /
// hash3 heads need (stream, hash) order, BinTree.java:170-207), so the stream
// bits never need digit passes: each stream is its own segment, sorted by one
// workgroup that walks it tile by tile and keeps the running bucket bases in
// LDS (no cross-workgroup scan). Per pass and item: one 8-byte read and one
// 8-byte write (the first pass reads the key and the position, the last
// writes them back in the match finder's layout).
//   seg_hist_kernel   one read sweep: every pass's digit histogram per stream
//   seg_pass_kernel   one digit pass: per tile of 2048 items, each wave ranks
//                     its 8 rounds of 64 items by wave-level multi-split (one
//                     ballot per digit bit gives the lanes with the same digit;
//                     the rank is their count below the lane), the waves'
//                     counts are scanned, the tile is sorted into LDS and then
//                     written out in that order, so a bucket's items leave as
//                     contiguous runs
// Items in flight are packed u64: hash bits | sentinel << 31 in the high word,
// the global position in the low word. Sentinel keys (positions that insert
// nothing, BinTree.java:153-162) sort after every real key of their stream, as
// they do in the full-key order.
#include "lzma_common.h"
#include "runtime.h"

namespace lzg {

constexpr int kSW = 64;                  // ballot group (hardware wave) size
constexpr int kSortThreads = 256;
constexpr int kSortWaves = kSortThreads / kSW;
#ifndef LZG_SORT_ROUNDS
#define LZG_SORT_ROUNDS 8
#endif
constexpr int kSortRounds = LZG_SORT_ROUNDS;   // rounds of kSW items per wave and tile
constexpr int kSortTile = kSortThreads * kSortRounds;
constexpr int kMaxPasses = 4;

enum { SK_PACKED = 0, SK_KEY64 = 1, SK_KEY32 = 2 };
constexpr size_t kHistLds = (size_t)kSortWaves * kMaxPasses * 256 * 4;
constexpr size_t kPassLds = (size_t)kSortTile * 8 + 4 * 256 * 4 + (size_t)kSortWaves * 256 * 4;

// One long segment (a single stream: config 4's 1 GiB stream, the JNI single-stream path)
// would leave all but one workgroup idle, so it is cut into chunks of kChunk items, one
// workgroup each: per pass, a histogram per chunk of that pass's input (chunk_hist_kernel),
// a scan over the chunks giving each chunk's bucket bases (chunk_scan_kernel), then the same
// tile pass per chunk. Stable: the chunks are in position order and each is ranked in order.
constexpr uint64_t kChunk = 1u << 16;

struct SortPass {
    const void* kin;          // SK_KEY64 / SK_KEY32 keys, or packed items (SK_PACKED)
    const uint32_t* vin;      // values (first pass only); null: each item's own index
    void* kout;               // packed items, or the final keys
    uint32_t* vout;           // final positions (last pass only)
    const uint64_t* offs;     // stream offsets (nstreams + 1), relative to the pass
    const uint64_t* ends;     // segment ends (segment s = [offs[s], ends[s])), or null: offs[s + 1]
    const uint64_t* dofs;     // where the last pass writes segment s (compaction), or null: offs[s]
    const uint32_t* hist;     // [nstreams][kMaxPasses][256]
    uint32_t pass, shift, bits, end_bit;
    const uint32_t* cbase;    // chunked (one segment): bucket bases per chunk [nchunks][256], else null
};

__device__ __forceinline__ uint32_t lanemask_count(uint64_t m) {   // set bits of m below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <int IN>
__device__ __forceinline__ uint64_t load_item(const SortPass& a, uint64_t i, uint32_t end_bit) {
    const uint32_t mask = end_bit >= 32 ? ~0u : ((1u << end_bit) - 1);
    if (IN == SK_PACKED) return ((const uint64_t*)a.kin)[i];
    uint32_t h, sent;
    if (IN == SK_KEY64) {
        const uint64_t k = ((const uint64_t*)a.kin)[i];
        sent = k == ~0ull;
        h = (uint32_t)k & mask;
    } else {
        const uint32_t k = ((const uint32_t*)a.kin)[i];
        sent = k == ~0u;
        h = k & mask;
    }
    return ((uint64_t)(h | (sent << 31)) << 32) | (a.vin ? a.vin[i] : (uint32_t)i);   // no vin: the index
}

// every pass's histogram of one stream (one read sweep); per-wave LDS copies keep
// the atomics of different waves apart
template <int IN>
__global__ void __launch_bounds__(kSortThreads) seg_hist_kernel(SortPass a, uint32_t npass, uint32_t widths,
                                                                 uint32_t* __restrict__ hist) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];   // dynamic LDS (the CPU emulation shares it)
    auto h = (uint32_t(*)[kMaxPasses][256])smem;                        // [kSortWaves][kMaxPasses][256]
    const uint32_t tid = threadIdx.x, w = tid / kSW;
    for (uint32_t k = tid; k < kSortWaves * kMaxPasses * 256; k += kSortThreads) (&h[0][0][0])[k] = 0;
    __syncthreads();
    const uint32_t s = blockIdx.x;
    const uint64_t lo = a.offs[s], n = (a.ends ? a.ends[s] : a.offs[s + 1]) - lo;
    for (uint64_t i = tid; i < n; i += kSortThreads) {
        const uint64_t it = load_item<IN>(a, lo + i, a.end_bit);
        const uint32_t hb = (uint32_t)(it >> 32) & 0x7FFFFFFFu;
        uint32_t sh = 0;
        for (uint32_t p = 0; p < npass; p++) {
            const uint32_t b = (widths >> (4 * p)) & 15u;   // pass p's digit width
            atomicAdd(&h[w][p][(hb >> sh) & ((1u << b) - 1)], 1u);
            sh += b;
        }
    }
    __syncthreads();
    for (uint32_t k = tid; k < kMaxPasses * 256; k += kSortThreads) {
        uint32_t v = 0;
        for (int x = 0; x < kSortWaves; x++) v += (&h[x][0][0])[k];
        hist[(size_t)s * kMaxPasses * 256 + k] = v;
    }
}

// the chunked form's histograms: chunk c of segment 0 (this pass's input order), one digit
template <int IN>
__global__ void __launch_bounds__(kSortThreads) chunk_hist_kernel(SortPass a, uint32_t* __restrict__ chist) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];   // dynamic LDS (the CPU emulation shares it)
    auto h = (uint32_t(*)[256])smem;                                    // [kSortWaves][256]
    const uint32_t tid = threadIdx.x, w = tid / kSW;
    for (uint32_t k = tid; k < kSortWaves * 256; k += kSortThreads) (&h[0][0])[k] = 0;
    __syncthreads();
    const uint64_t seg_lo = a.offs[0], seg_hi = a.ends ? a.ends[0] : a.offs[1];
    const uint64_t lo = seg_lo + (uint64_t)blockIdx.x * kChunk;
    const uint64_t n = lo >= seg_hi ? 0 : (seg_hi - lo < kChunk ? seg_hi - lo : kChunk);
    const uint32_t dmask = (1u << a.bits) - 1;
    for (uint64_t i = tid; i < n; i += kSortThreads) {
        const uint64_t it = load_item<IN>(a, lo + i, a.end_bit);
        atomicAdd(&h[w][(uint32_t)(it >> (32 + a.shift)) & dmask], 1u);
    }
    __syncthreads();
    uint32_t v = 0;
    for (int x = 0; x < kSortWaves; x++) v += h[x][tid];
    chist[(size_t)blockIdx.x * 256 + tid] = v;
}

// chunk c's bucket bases: digit d's start in the segment (the counts of smaller digits)
// plus the counts of digit d in chunks before c; one thread per digit
__global__ void __launch_bounds__(256) chunk_scan_kernel(uint32_t* __restrict__ chist, uint32_t nchunks) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];   // dynamic LDS (the CPU emulation shares it)
    uint32_t* scan = (uint32_t*)smem;                                   // [256]
    const uint32_t d = threadIdx.x;
    uint32_t run = 0;
    for (uint32_t c = 0; c < nchunks; c++) {
        const uint32_t v = chist[(size_t)c * 256 + d];
        chist[(size_t)c * 256 + d] = run;
        run += v;
    }
    scan[d] = run;
    __syncthreads();
    for (uint32_t o = 1; o < 256; o <<= 1) {
        const uint32_t v = d >= o ? scan[d - o] : 0u;
        __syncthreads();
        scan[d] += v;
        __syncthreads();
    }
    const uint32_t base = scan[d] - run;   // the digits below d, over the whole segment
    for (uint32_t c = 0; c < nchunks; c++) chist[(size_t)c * 256 + d] += base;
}

template <int IN, int OUT>
__global__ void __launch_bounds__(kSortThreads) seg_pass_kernel(SortPass a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];   // dynamic LDS (the CPU emulation shares it)
    uint64_t* tile = (uint64_t*)smem;                                   // [kSortTile]
    uint32_t* base = (uint32_t*)(tile + kSortTile);
    uint32_t* tot = base + 256;
    uint32_t* loff = tot + 256;
    uint32_t* scan = loff + 256;
    auto cnt = (uint32_t(*)[256])(scan + 256);                           // [kSortWaves][256]
    const uint32_t tid = threadIdx.x, w = tid / kSW, lane = tid % kSW;
    const uint32_t s = a.cbase ? 0u : blockIdx.x;
    const uint64_t seg_lo = a.offs[s], seg_hi = a.ends ? a.ends[s] : a.offs[s + 1];
    uint64_t lo = seg_lo, n = seg_hi - seg_lo;
    if (a.cbase) {   // chunked: this block's chunk of segment 0, its bases from chunk_scan_kernel
        lo = seg_lo + (uint64_t)blockIdx.x * kChunk;
        if (lo >= seg_hi) return;   // the whole block: past the segment's end
        n = seg_hi - lo < kChunk ? seg_hi - lo : kChunk;
    }
    const uint32_t nb = 1u << a.bits, dmask = nb - 1;
    if (a.cbase) {
        base[tid] = a.cbase[(size_t)blockIdx.x * 256 + tid];
    } else {
        // bucket bases of this stream: exclusive scan of its histogram (Hillis-Steele in LDS)
        const uint32_t hv = tid < nb ? a.hist[((size_t)s * kMaxPasses + a.pass) * 256 + tid] : 0u;
        scan[tid] = hv;
        __syncthreads();
        for (uint32_t o = 1; o < 256; o <<= 1) {
            const uint32_t v = tid >= o ? scan[tid - o] : 0u;
            __syncthreads();
            scan[tid] += v;
            __syncthreads();
        }
        base[tid] = scan[tid] - hv;
    }
    for (uint32_t x = 0; x < kSortWaves; x++) cnt[x][tid] = 0;
    __syncthreads();
    for (uint64_t t0 = 0; t0 < n; t0 += kSortTile) {
        const uint32_t tn = n - t0 < (uint64_t)kSortTile ? (uint32_t)(n - t0) : (uint32_t)kSortTile;
        uint64_t item[kSortRounds];
        uint32_t dig[kSortRounds], rank[kSortRounds];
#pragma unroll
        for (int r = 0; r < kSortRounds; r++) {
            const uint32_t k = w * (kSW * kSortRounds) + r * kSW + lane;   // this wave's contiguous 512 items
            item[r] = k < tn ? load_item<IN>(a, lo + t0 + k, a.end_bit) : 0ull;
            dig[r] = (uint32_t)(item[r] >> (32 + a.shift)) & dmask;
        }
        // wave-level multi-split: lanes with this lane's digit, rank = their count below
        // the lane plus the wave's earlier count of the digit (cnt[w][d], in LDS)
#pragma unroll
        for (int r = 0; r < kSortRounds; r++) {
            const uint32_t k = w * (kSW * kSortRounds) + r * kSW + lane;
            const bool valid = k < tn;
            uint64_t peers = __ballot(valid);
            for (uint32_t b = 0; b < a.bits; b++) {
                const bool on = (dig[r] >> b) & 1u;
                const uint64_t m = __ballot(on);
                peers &= on ? m : ~m;
            }
            const uint32_t below = lanemask_count(peers);
            const uint32_t before = valid ? cnt[w][dig[r]] : 0u;
            rank[r] = before + below;
            __builtin_amdgcn_wave_barrier();
            if (valid && below == 0) cnt[w][dig[r]] = before + (uint32_t)__builtin_popcountll(peers);
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
        // per digit: exclusive offsets of the waves, the tile total, the tile-local start
        {
            uint32_t run = 0;
            for (uint32_t x = 0; x < kSortWaves; x++) { const uint32_t c = cnt[x][tid]; cnt[x][tid] = run; run += c; }
            tot[tid] = run;
            scan[tid] = run;
        }
        __syncthreads();
        for (uint32_t o = 1; o < 256; o <<= 1) {
            const uint32_t v = tid >= o ? scan[tid - o] : 0u;
            __syncthreads();
            scan[tid] += v;
            __syncthreads();
        }
        loff[tid] = scan[tid] - tot[tid];
        __syncthreads();
#pragma unroll
        for (int r = 0; r < kSortRounds; r++) {
            const uint32_t k = w * (kSW * kSortRounds) + r * kSW + lane;
            if (k < tn) tile[loff[dig[r]] + cnt[w][dig[r]] + rank[r]] = item[r];
        }
        __syncthreads();
        for (uint32_t j = tid; j < tn; j += kSortThreads) {
            const uint64_t it = tile[j];
            const uint32_t d = (uint32_t)(it >> (32 + a.shift)) & dmask;
            const uint64_t dst = (OUT != SK_PACKED && a.dofs ? a.dofs[s] : seg_lo) + base[d] + (j - loff[d]);
            if (OUT == SK_PACKED) {
                ((uint64_t*)a.kout)[dst] = it;
            } else {
                const uint32_t hi = (uint32_t)(it >> 32);
                const bool sent = (hi >> 31) != 0;
                const uint32_t h = hi & 0x7FFFFFFFu;
                if (OUT == SK_KEY64) ((uint64_t*)a.kout)[dst] = sent ? ~0ull : (((uint64_t)s << a.end_bit) | h);
                else ((uint32_t*)a.kout)[dst] = sent ? ~0u : ((s << a.end_bit) | h);
                a.vout[dst] = (uint32_t)it;
            }
        }
        __syncthreads();
        base[tid] += tot[tid];
        for (uint32_t x = 0; x < kSortWaves; x++) cnt[x][tid] = 0;
        __syncthreads();
    }
}

template <int IN, int OUT>
static void launch_pass(const SortPass& p, int nblocks, hipStream_t st, uint32_t* chist) {
    if (p.cbase) {   // chunked: this pass's per-chunk histograms and bases first
        hipLaunchKernelGGL((chunk_hist_kernel<IN>), dim3(nblocks), dim3(kSortThreads), (size_t)kSortWaves * 256 * 4, st, p, chist);
        hipLaunchKernelGGL(chunk_scan_kernel, dim3(1), dim3(256), 256 * 4, st, chist, (uint32_t)nblocks);
    }
    hipLaunchKernelGGL((seg_pass_kernel<IN, OUT>), dim3(nblocks), dim3(kSortThreads), kPassLds, st, p);
}

// Stable sort of every stream's items by the low end_bit bits of their keys.
// key64: keys are u64 (else u32); tmp_a / tmp_b: n u64 each; hist: nstreams * 1024 u32.
// d_ends (optional): segment s is [offs[s], ends[s]); d_dofs (optional): the sorted
// segment s is written from d_dofs[s] on (the segments compacted into one list).
int seg_radix_sort(Ctx* ctx, bool key64, const void* kin, const uint32_t* vin, void* kout, uint32_t* vout,
                   uint64_t* tmp_a, uint64_t* tmp_b, uint32_t* hist, uint64_t n, const uint64_t* d_offs, int nstreams,
                   int end_bit, hipStream_t st, const uint64_t* d_ends, const uint64_t* d_dofs) {
    if (n == 0 || nstreams <= 0) return LZMA_OK;
    if (end_bit < 1 || end_bit > 31) return ctx->fail(LZMA_E_INTERNAL, "seg_radix_sort: %d key bits", end_bit);
    const uint32_t npass = (uint32_t)(end_bit + 7) / 8;
    if (npass > (uint32_t)kMaxPasses) return ctx->fail(LZMA_E_INTERNAL, "seg_radix_sort: %u passes", npass);
    // digit widths <= 8: the first end_bit % npass passes take one bit more
    uint32_t width[kMaxPasses] = {0, 0, 0, 0}, widths = 0;
    for (uint32_t q = 0; q < npass; q++) {
        width[q] = (uint32_t)end_bit / npass + (q < (uint32_t)end_bit % npass ? 1u : 0u);
        widths |= width[q] << (4 * q);
        if (width[q] > 8) return ctx->fail(LZMA_E_INTERNAL, "seg_radix_sort: %u-bit digit", width[q]);   // LDS tables hold 256
    }
    SortPass p{};
    p.kin = kin; p.vin = vin; p.offs = d_offs; p.ends = d_ends; p.dofs = d_dofs; p.hist = hist; p.end_bit = (uint32_t)end_bit;
    // one long segment: chunked (n bounds the segment; blocks past its end exit), the chunk
    // histograms and bases in `hist` (sort_hist_words)
    const bool chunked = nstreams == 1 && n > 4 * kChunk;
    const int nblocks = chunked ? (int)((n + kChunk - 1) / kChunk) : nstreams;
    if (chunked) {
        p.cbase = hist;
    } else if (key64) {
        hipLaunchKernelGGL((seg_hist_kernel<SK_KEY64>), dim3(nstreams), dim3(kSortThreads), kHistLds, st, p, npass, widths, hist);
    } else {
        hipLaunchKernelGGL((seg_hist_kernel<SK_KEY32>), dim3(nstreams), dim3(kSortThreads), kHistLds, st, p, npass, widths, hist);
    }
    uint32_t shift = 0;
    uint64_t* bufs[2] = {tmp_a, tmp_b};
    for (uint32_t q = 0; q < npass; q++) {
        SortPass x = p;
        x.pass = q;
        x.shift = shift;
        x.bits = width[q];
        const bool first = q == 0, last = q + 1 == npass;
        x.kin = first ? kin : (const void*)bufs[(q + 1) & 1];
        x.kout = last ? kout : (void*)bufs[q & 1];
        x.vout = vout;
        const int in = first ? (key64 ? SK_KEY64 : SK_KEY32) : SK_PACKED;
        const int out = last ? (key64 ? SK_KEY64 : SK_KEY32) : SK_PACKED;
        uint32_t* ch = chunked ? hist : nullptr;
        if (in == SK_KEY64 && out == SK_KEY64) launch_pass<SK_KEY64, SK_KEY64>(x, nblocks, st, ch);
        else if (in == SK_KEY64) launch_pass<SK_KEY64, SK_PACKED>(x, nblocks, st, ch);
        else if (in == SK_KEY32 && out == SK_KEY32) launch_pass<SK_KEY32, SK_KEY32>(x, nblocks, st, ch);
        else if (in == SK_KEY32) launch_pass<SK_KEY32, SK_PACKED>(x, nblocks, st, ch);
        else if (out == SK_KEY64) launch_pass<SK_PACKED, SK_KEY64>(x, nblocks, st, ch);
        else if (out == SK_KEY32) launch_pass<SK_PACKED, SK_KEY32>(x, nblocks, st, ch);
        else launch_pass<SK_PACKED, SK_PACKED>(x, nblocks, st, ch);
        shift += x.bits;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return ctx->fail(LZMA_E_DEVICE, "seg_radix_sort: %s", hipGetErrorString(e));
    return LZMA_OK;
}

// u32 words the `hist` argument of seg_radix_sort needs: every pass's histogram per stream,
// or, for one long segment (chunked), the bases of every chunk
size_t sort_hist_words(uint64_t n, int nstreams) {
    const size_t seg = (size_t)nstreams * kMaxPasses * 256;
    const size_t chunked = nstreams == 1 ? (size_t)((n + kChunk - 1) / kChunk) * 256 : 0;
    return seg > chunked ? seg : chunked;
}

}  // namespace lzg
