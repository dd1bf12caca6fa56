/*
 * oracle_cli.c -- TEST INFRASTRUCTURE ONLY. LzmaAlone-style front end
 * (LzmaAlone.java:156-248) over the C restatement, used to check the
 * reference's golden .lzma md5s: `oracle_cli e [-d N -fb N -lc N -lp N -pb N
 * -mfbt2|-mfbt4 -eos] in out` and `oracle_cli d in out`.
 */
#include "lzma_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static unsigned char *slurp(const char *path, long *n) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END); *n = ftell(f); fseek(f, 0, SEEK_SET);
    unsigned char *b = malloc(*n + 1);
    if (fread(b, 1, *n, f) != (size_t)*n) { fclose(f); free(b); return NULL; }
    fclose(f);
    return b;
}

int main(int argc, char **argv) {
    if (argc < 4) { fprintf(stderr, "usage: %s e|d [switches] in out\n", argv[0]); return 2; }
    oracle_params p = { 1 << 23, 128, 1, 3, 0, 2, 0 };   /* LzmaAlone.java:24-37 */
    int enc = strcmp(argv[1], "e") == 0;
    int i;
    for (i = 2; i < argc - 2; i++) {
        const char *s = argv[i] + 1;
        if (!strncmp(s, "fb", 2)) p.fb = atoi(s + 2);
        else if (!strncmp(s, "lc", 2)) p.lc = atoi(s + 2);
        else if (!strncmp(s, "lp", 2)) p.lp = atoi(s + 2);
        else if (!strncmp(s, "pb", 2)) p.pb = atoi(s + 2);
        else if (!strcmp(s, "eos")) p.eos = 1;
        else if (!strcmp(s, "mfbt2")) p.mf = 0;
        else if (!strcmp(s, "mfbt4")) p.mf = 1;
        else if (!strcmp(s, "mfbt4b")) p.mf = 2;
        else if (s[0] == 'd') p.dict_size = 1 << atoi(s + 1);
        else { fprintf(stderr, "bad switch %s\n", argv[i]); return 2; }
    }
    long n;
    unsigned char *in = slurp(argv[argc - 2], &n);
    if (!in) { perror("read"); return 1; }
    FILE *fo = fopen(argv[argc - 1], "wb");
    if (enc) {
        unsigned char hdr[13];
        oracle_write_props(&p, hdr);
        long long sz = p.eos ? -1 : n;
        for (int k = 0; k < 8; k++) hdr[5 + k] = (unsigned char)((unsigned long long)sz >> (8 * k));
        unsigned char *out; unsigned long long ol;
        if (oracle_encode(in, n, &p, 0, &out, (uint64_t *)&ol) != 0) { fprintf(stderr, "encode failed\n"); return 1; }
        fwrite(hdr, 1, 13, fo); fwrite(out, 1, ol, fo);
        oracle_free(out);
    } else {
        long long sz = 0;
        for (int k = 0; k < 8; k++) sz |= (long long)in[5 + k] << (8 * k);
        unsigned long long cap = sz >= 0 ? (unsigned long long)sz + 1024 : (unsigned long long)n * 64 + (1 << 20);
        unsigned char *out = malloc(cap);
        unsigned long long ol;
        int rc = oracle_decode(in + 13, n - 13, in, sz, out, cap, (uint64_t *)&ol);
        if (rc != 1) { fprintf(stderr, "decode failed %d\n", rc); return 1; }
        fwrite(out, 1, ol, fo);
        free(out);
    }
    fclose(fo);
    free(in);
    return 0;
}
