/*
 * lzma_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference LZMA encoder/decoder (rfalke/lzma-java,
 * a Java port of the 7-Zip LZMA SDK 4.61). It is the parity checker for the
 * MI355X product path: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product library never links it.
 *
 * Parity pinning: the restatement reproduces the 12 md5/length golden
 * vectors of src/test/java/SevenZip/LzmaAloneTest.java:27-38 on firefox.exe,
 * the range-coder known answers of
 * src/test/java/SevenZip/Compression/RangeCoder/EncoderLearningTest.java:29-73
 * and the bit-tree prices of BitTreeEncoderLearningTest.java:24-31
 * (see tests/test_oracle.py). The reference itself (Java) cannot be built
 * here: no JDK exists in this container.
 */
#ifndef LZMA_ORACLE_H
#define LZMA_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_params {
    int32_t dict_size; /* Encoder.SetDictionarySize  (Encoder.java:1135) */
    int32_t fb;        /* Encoder.SetNumFastBytes    (Encoder.java:1148) */
    int32_t mf;        /* Encoder.SetMatchFinder 0=bt2 1=bt4 2=bt4b (Encoder.java:1156) */
    int32_t lc, lp, pb;/* Encoder.SetLcLpPb          (Encoder.java:1169) */
    int32_t eos;       /* Encoder.SetEndMarkerMode   (Encoder.java:1182) */
} oracle_params;

/* Encoder.WriteCoderProperties (Encoder.java:1079-1085). */
void oracle_write_props(const oracle_params *p, uint8_t out[5]);

/* Encoder.Code (Encoder.java:1064) on one in-memory stream: raw range-coder
 * bytes, no .lzma header. *out is malloc'd; caller frees with oracle_free.
 * mode 0 = reference call sequence (fillMatches / Skip as Encoder does);
 * mode 1 = two-phase: match lists precomputed for every position with
 * fillMatches, then the parser consumes them (checks that BT4 output does
 * not depend on parser decisions). Returns 0 on success. */
int oracle_encode(const uint8_t *in, uint64_t n, const oracle_params *p, int mode,
                  uint8_t **out, uint64_t *out_len);
void oracle_free(void *ptr);

/* Encoder session: one reused Encoder instance (its match-finder arrays are
 * kept across calls and the hash heads cleared per call, BinTree.java:72-80,
 * 108-133). oracle_enc_code's *out points into the session and stays valid
 * until the next call. Same bytes as oracle_encode(mode 0). */
typedef struct oracle_enc oracle_enc;
oracle_enc *oracle_enc_new(const oracle_params *p);
int oracle_enc_code(oracle_enc *s, const uint8_t *in, uint64_t n, const uint8_t **out, uint64_t *out_len);
void oracle_enc_delete(oracle_enc *s);

/* Decoder.SetDecoderProperties + Decoder.Code (Decoder.java:205-318).
 * out_size < 0 => decode until end marker. Returns 1 on success (Java true),
 * 0 on a corrupt stream (Java false), -1 on output overflow / bad props. */
int oracle_decode(const uint8_t *in, uint64_t n_in, const uint8_t props[5], int64_t out_size,
                  uint8_t *out, uint64_t out_cap, uint64_t *out_len);

/* Match lists for every position (BinTree.fillMatches at all positions,
 * BinTree.java:152-273), plus the ReadMatchDistances extension of the
 * longest pair (Encoder.java:275-287). counts[n], main_len[n]; pairs packed
 * (len, dist) into lens/dists, at most cap entries. Returns total pairs or -1. */
int64_t oracle_match_lists(const uint8_t *in, uint64_t n, const oracle_params *p,
                           uint32_t *counts, uint32_t *main_len,
                           uint32_t *lens, uint32_t *dists, uint64_t cap);

/* Known-answer hooks for RangeEncoder / BitTreeEncoder unit tests. */
int oracle_rc_encode_bits(const int32_t *bits, int n, uint8_t *out, int cap);
int oracle_rc_direct_bits(const uint32_t *vals, const int32_t *nbits, int n, uint8_t *out, int cap);
void oracle_bittree_prices_after(int num_bit_levels, int encoded_symbol, uint32_t *prices);
uint32_t oracle_prob_price(int index);
/* Normalize calls so far (BinTree.java:358-375; the `norm` test build lowers its threshold) */
uint64_t oracle_normalize_count(void);

#ifdef __cplusplus
}
#endif
#endif
