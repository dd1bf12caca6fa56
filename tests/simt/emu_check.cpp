// TEST INFRASTRUCTURE ONLY -- runs the product's C ABI (lzma-java_amd/csrc
// compiled against the CPU SIMT emulation headers) against the oracle, under
// AddressSanitizer. Usage: emu_check [quick|full]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <string>
#include <vector>

#include "../../include/lzma_mi355x.h"
#include "../../oracle/lzma_oracle.h"

namespace lzg { alignas(16) uint8_t smem[160 * 1024]; namespace sliced { alignas(16) uint8_t smem[160 * 1024]; } }

static std::vector<uint8_t> make_input(int kind, size_t n, unsigned seed) {
    std::vector<uint8_t> v(n);
    std::mt19937 rng(seed);
    switch (kind) {
        case 0: for (auto& x : v) x = (uint8_t)rng(); break;
        case 1: for (auto& x : v) x = (uint8_t)(rng() % 3); break;
        case 2: { const char* w[] = {"alpha", "beta", "gamma", " ", "the", "\n"}; size_t i = 0;
                  while (i < n) { const char* s = w[rng() % 6]; for (size_t k = 0; s[k] && i < n; k++) v[i++] = (uint8_t)s[k]; } break; }
        case 3: for (size_t i = 0; i < n; i++) v[i] = (uint8_t)("abcdefghij"[i % 10]); break;
        case 4: lzma_bench_generate(v.data(), n); break;
        case 6: lzma_text_generate(v.data(), n, seed); break;   // deep getOptimum parses (_optimum ring)
        default: if (n) memset(v.data(), 0, n);
    }
    return v;
}

int main(int argc, char** argv) {
    fprintf(stderr, "emu_check start\n");
    bool full = argc > 1 && !strcmp(argv[1], "full");
    bool tiny = argc > 1 && !strcmp(argv[1], "tiny");
    lzma_ctx* ctx = nullptr;
    if (lzma_ctx_create(0, &ctx) != LZMA_OK) { printf("ctx fail\n"); return 1; }
    struct P { lzma_params p; };
    std::vector<lzma_params> ps = {
        {1 << 26, 32, 1, 3, 0, 2, 0}, {1 << 12, 5, 0, 3, 0, 2, 0}, {1 << 20, 273, 1, 0, 2, 0, 0},
        {100, 64, 2, 3, 0, 2, 1}, {1, 16, 1, 3, 0, 2, 0}, {1 << 16, 48, 1, 8, 0, 4, 0}, {1 << 23, 128, 1, 3, 0, 2, 0},
    };
    int fails = 0, total = 0;
    std::vector<size_t> sizes = {0, 1, 2, 3, 4, 5, 17, 300, 3000};
    if (full) { sizes.push_back(20000); sizes.push_back(70000); }
    if (tiny) { sizes = {0, 1, 2, 5, 17, 300}; ps.resize(1); }
    for (size_t pi = 0; pi < ps.size(); pi++) {
        const lzma_params& p = ps[pi];
        oracle_params op = {p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos};
        std::vector<std::vector<uint8_t>> ins;
        for (int kind = 0; kind < (tiny ? 2 : 6); kind++)
            for (size_t n : sizes) ins.push_back(make_input(kind, n, (unsigned)(kind * 1000 + n + pi)));
        if (!tiny) ins.push_back(make_input(6, full ? 200000 : 40000, (unsigned)(7 + pi)));
        std::vector<uint64_t> offs(ins.size() + 1, 0);
        std::vector<uint8_t> cat;
        for (size_t i = 0; i < ins.size(); i++) { cat.insert(cat.end(), ins[i].begin(), ins[i].end()); offs[i + 1] = cat.size(); }
        uint64_t cap = 0;
        for (auto& x : ins) cap += lzma_enc_bound(x.size());
        std::vector<uint8_t> out(cap + 1);
        std::vector<uint64_t> oo(ins.size() + 1);
        int rc = lzma_enc_batch(ctx, &p, cat.data(), offs.data(), (int)ins.size(), out.data(), cap, oo.data());
        if (rc) { printf("param %zu: enc_batch rc=%d %s\n", pi, rc, lzma_last_error(ctx)); fails++; continue; }
        std::vector<uint8_t> props(5);
        lzma_write_props(&p, props.data());
        for (size_t i = 0; i < ins.size(); i++) {
            uint8_t* ref; uint64_t rl;
            oracle_encode(ins[i].data(), ins[i].size(), &op, 0, &ref, &rl);
            uint64_t gl = oo[i + 1] - oo[i];
            total++;
            bool ok = gl == rl && !memcmp(out.data() + oo[i], ref, rl);
            if (!ok) {
                fails++;
                uint64_t k = 0;
                while (k < gl && k < rl && out[oo[i] + k] == ref[k]) k++;
                printf("MISMATCH param %zu stream %zu (n=%zu kind=%zu): gpu %llu ref %llu bytes, first diff at %llu\n", pi, i,
                       ins[i].size(), i / sizes.size(), (unsigned long long)gl, (unsigned long long)rl, (unsigned long long)k);
            } else {
                // decode back through the emulated decoder
                std::vector<uint8_t> dec(ins[i].size() + 64);
                uint64_t dl = 0;
                int drc = lzma_decode(ctx, props.data(), ref, rl, p.eos ? -1 : (int64_t)ins[i].size(), dec.data(), dec.size(), &dl);
                if (drc != LZMA_OK || dl != ins[i].size() || memcmp(dec.data(), ins[i].data(), dl)) {
                    fails++;
                    printf("DECODE FAIL param %zu stream %zu rc=%d len %llu\n", pi, i, drc, (unsigned long long)dl);
                }
            }
            oracle_free(ref);
        }
        printf("param %zu done\n", pi);
        fflush(stdout);
    }
    printf("%d/%d streams bit-exact, %d failures\n", total - fails, total, fails);
    lzma_ctx_destroy(ctx);
    return fails ? 1 : 0;
}
