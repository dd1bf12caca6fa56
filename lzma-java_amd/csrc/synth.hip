// synth.hip -- the synthetic inputs of SURVEY.md 8(d) besides the LzmaBench
// generator (runtime.hip): RND (config 1) and TEXT (config 3). Host code only;
// exported through the C ABI so bench.py, the tests and a Java harness all
// draw the same bytes.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/lzma_mi355x.h"

namespace {

inline uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

constexpr int kVocab = 50000;

// The fixed vocabulary: word lengths and letters drawn from English-like
// weights with a constant seed (only the word draws depend on the caller's seed).
struct Vocab {
    std::vector<uint32_t> off;
    std::vector<char> chars;
    std::vector<double> cdf;   // Zipf(s = 1.1) over ranks 1..kVocab, unnormalised
    static constexpr int kGuide = 1 << 16;
    std::vector<uint32_t> guide;   // guide[k] = first rank whose cdf exceeds k / kGuide of the total
    Vocab() {
        static const uint16_t letter_w[26] = {82, 15, 28, 43, 127, 22, 20, 61, 70, 2, 8, 40, 24,
                                              67, 75, 19, 1, 60, 63, 91, 28, 10, 24, 2, 20, 1};
        static const uint16_t len_w[14] = {30, 170, 210, 160, 110, 90, 80, 60, 40, 20, 10, 10, 5, 5};
        uint32_t lcum[26], lsum = 0, ncum[14], nsum = 0;
        for (int i = 0; i < 26; i++) lcum[i] = (lsum += letter_w[i]);
        for (int i = 0; i < 14; i++) ncum[i] = (nsum += len_w[i]);
        uint64_t vx = 0x7E57ull;
        off.resize(kVocab + 1);
        chars.reserve(kVocab * 8);
        for (int w = 0; w < kVocab; w++) {
            off[w] = (uint32_t)chars.size();
            uint32_t r = (uint32_t)(splitmix64(vx) % nsum), len = 1;
            while (ncum[len - 1] <= r) len++;
            if (w >= 200 && len < 3) len += 2;   // only the most frequent words are very short
            for (uint32_t k = 0; k < len; k++) {
                uint32_t q = (uint32_t)(splitmix64(vx) % lsum), c = 0;
                while (lcum[c] <= q) c++;
                chars.push_back((char)('a' + c));
            }
        }
        off[kVocab] = (uint32_t)chars.size();
        cdf.resize(kVocab);
        double acc = 0;
        for (int r = 0; r < kVocab; r++) cdf[r] = (acc += 1.0 / std::pow((double)(r + 1), 1.1));
        guide.resize(kGuide + 1);
        for (int k = 0, r = 0; k <= kGuide; k++) {
            const double u = acc * (double)k / kGuide;
            while (r < kVocab - 1 && cdf[r] <= u) r++;
            guide[k] = (uint32_t)r;
        }
    }
};

struct TextWriter {
    const Vocab& v;
    uint8_t* buf;
    uint64_t size, pos = 0;
    uint64_t x;
    TextWriter(const Vocab& vv, uint8_t* b, uint64_t n, uint64_t seed) : v(vv), buf(b), size(n), x(seed) {}
    uint32_t below(uint32_t n) { return (uint32_t)(splitmix64(x) % n); }
    int draw() {
        const double f = (double)(splitmix64(x) >> 11) * (1.0 / 9007199254740992.0);
        const double u = f * v.cdf.back();
        const size_t k = (size_t)(f * Vocab::kGuide);
        // the answer lies in [guide[k], guide[k + 1]]: upper_bound over that bracket
        auto lo = v.cdf.begin() + v.guide[k], hi = v.cdf.begin() + v.guide[k + 1] + 1;
        const int r = (int)(std::upper_bound(lo, hi, u) - v.cdf.begin());
        return r < kVocab ? r : kVocab - 1;
    }
    void put(const char* s, size_t n) {
        for (size_t k = 0; k < n && pos < size; k++) buf[pos++] = (uint8_t)s[k];
    }
    void put(const char* s) { put(s, strlen(s)); }
    void word(int w, bool cap) {
        const char* s = &v.chars[v.off[w]];
        size_t n = v.off[w + 1] - v.off[w];
        if (cap && n && pos < size) { buf[pos++] = (uint8_t)(s[0] - 'a' + 'A'); s++; n--; }
        put(s, n);
    }
    void words(uint32_t n, bool cap_first) {
        for (uint32_t k = 0; k < n; k++) {
            if (k) put(" ");
            word(draw(), cap_first && k == 0);
        }
    }
    void markup(bool& sentence_start) {
        char num[64];
        switch (below(7)) {
            case 0:   // section heading
                put("\n\n== ");
                for (uint32_t k = 0, nw = 1 + below(4); k < nw; k++) { if (k) put(" "); word(draw(), true); }
                put(" ==\n");
                sentence_start = true;
                break;
            case 1: put("[["); word(draw(), false); put("]] "); break;
            case 2: put("[["); word(draw(), false); put("|"); words(2, false); put("]] "); break;
            case 3: put("'''"); word(draw(), false); put("''' "); break;
            case 4:
                put("{{cite web |title=");
                words(2 + below(5), true);
                snprintf(num, sizeof num, " |year=%u |page=%u}} ", 1900 + below(125), 1 + below(900));
                put(num);
                break;
            case 5: put("<ref>"); words(3 + below(8), true); put(".</ref> "); break;
            default: put("\n* "); sentence_start = true; break;
        }
    }
    void run() {
        uint32_t until_markup = 150 + below(100);
        bool sentence_start = true;
        uint32_t sentence_left = 6 + below(19);
        while (pos < size) {
            if (until_markup-- == 0) {
                until_markup = 150 + below(100);
                markup(sentence_start);
                continue;
            }
            word(draw(), sentence_start);
            sentence_start = false;
            if (--sentence_left == 0) {
                put(below(8) == 0 ? ".\n" : ". ");
                sentence_start = true;
                sentence_left = 6 + below(19);
            } else {
                put(below(10) == 0 ? ", " : " ");
            }
        }
    }
};

}  // namespace

extern "C" {

void lzma_rnd_generate(uint8_t* buf, uint64_t size, uint64_t seed) {
    uint64_t x = seed, i = 0;
    for (; i + 8 <= size; i += 8) {
        const uint64_t v = splitmix64(x);
        for (int k = 0; k < 8; k++) buf[i + k] = (uint8_t)(v >> (8 * k));
    }
    if (i < size) {
        const uint64_t v = splitmix64(x);
        for (int k = 0; i < size; k++, i++) buf[i] = (uint8_t)(v >> (8 * k));
    }
}

void lzma_text_generate(uint8_t* buf, uint64_t size, uint64_t seed) {
    static const Vocab vocab;
    // independent 4 MiB segments, each from its own seed, generated in parallel:
    // the bytes depend only on (size, seed), not on the thread count
    constexpr uint64_t kSeg = 4ull << 20;
    const uint64_t nseg = (size + kSeg - 1) / kSeg;
    const unsigned nth = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(nseg, 16));
    std::atomic<uint64_t> next{0};
    auto work = [&]() {
        for (uint64_t k; (k = next.fetch_add(1)) < nseg;) {
            uint64_t sx = seed ^ (k * 0xD1B54A32D192ED03ull);
            const uint64_t a = k * kSeg, n = std::min(kSeg, size - a);
            TextWriter w(vocab, buf + a, n, splitmix64(sx));
            w.run();
        }
    };
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nth; t++) th.emplace_back(work);
    work();
    for (auto& t : th) t.join();
}

}  // extern "C"
