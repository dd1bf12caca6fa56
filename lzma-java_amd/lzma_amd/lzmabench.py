"""LzmaBench harness on the MI355X path.

Restates src/main/java/SevenZip/LzmaBench.java:226-403 (`LzmaAlone b [passes]
-dN`, LzmaAlone.java:170-178): the same CBenchRandomGenerator buffer of
dictionarySize + 2^21 bytes, Encoder defaults with the given dictionary, one
encode and two decodes per pass with a CRC check, and the same printed lines
and ratings (KB/s and the "MIPS" estimates of GetCompressRating /
GetDecompressRating).

Differences, both in what is timed, never in the bytes:
  * the reference starts its encode clock once dictionarySize input bytes have
    been consumed (CProgressInfo, LzmaBench.java:207-222, 366-367); the GPU
    encoder has no mid-stream progress callback, so the whole buffer is timed
    and benchSize = kBufferSize;
  * `copies` > 1 encodes that many identical independent streams per pass (one
    wavefront each) and counts all their bytes: the reference's single stream is
    copies = 1.
Device-resident buffers (the analogue of the reference's in-memory streams).
"""
import sys
import time
import zlib

import numpy as np

K_SUB_BITS = 8                      # LzmaBench.java:226
K_ADDITIONAL_SIZE = 1 << 21         # LzmaBench.java:12


def get_log_size(size: int) -> int:   # LzmaBench.java:228-237
    for i in range(K_SUB_BITS, 32):
        for j in range(1 << K_SUB_BITS):
            if size <= (1 << i) + (j << (i - K_SUB_BITS)):
                return (i << K_SUB_BITS) + j
    return 32 << K_SUB_BITS


def my_mult_div64(value: int, elapsed_ms: int) -> int:   # LzmaBench.java:239-250
    freq, el = 1000, elapsed_ms
    while freq > 1000000:
        freq >>= 1
        el >>= 1
    if el == 0:
        el = 1
    return value * freq // el


def get_compress_rating(dictionary_size: int, elapsed_ms: int, size: int) -> int:   # :252-257
    t = get_log_size(dictionary_size) - (18 << K_SUB_BITS)
    num_commands_for_one = 1060 + ((t * t * 10) >> (2 * K_SUB_BITS))
    return my_mult_div64(size * num_commands_for_one, elapsed_ms)


def get_decompress_rating(elapsed_ms: int, out_size: int, in_size: int) -> int:   # :259-262
    return my_mult_div64(in_size * 220 + out_size * 20, elapsed_ms)


def _value(v: int) -> str:   # PrintValue, :272-279
    return str(v).rjust(6)


def results(dictionary_size: int, elapsed_ms: int, size: int, decompress: bool, second_size: int) -> str:
    """PrintResults (LzmaBench.java:286-301) as a string."""
    speed = my_mult_div64(size, elapsed_ms)
    if decompress:
        rating = get_decompress_rating(elapsed_ms, size, second_size)
    else:
        rating = get_compress_rating(dictionary_size, elapsed_ms, size)
    return _value(speed // 1024) + " KB/s  " + _value(rating // 1000000) + " MIPS"


def lzma_benchmark(num_iterations: int, dictionary_size: int, ctx=None, out=sys.stdout, copies: int = 1) -> int:
    """LzmaBench.LzmaBenchmark (LzmaBench.java:303-403). Returns 0, or 1 for a too small dictionary."""
    import torch   # device buffers
    from . import Context, bench_generate, enc_bound, make_params, write_props

    if num_iterations <= 0:
        return 0
    if dictionary_size < (1 << 18):
        out.write("\nError: dictionary size for benchmark must be >= 18 (256 KB)\n")
        return 1
    out.write("\n       Compressing                Decompressing\n\n")
    p = make_params(dict_size=dictionary_size)   # Encoder defaults otherwise (Encoder.java:135-172)
    props = write_props(p)
    buf_size = dictionary_size + K_ADDITIONAL_SIZE
    data = bench_generate(buf_size)
    crc = zlib.crc32(data.tobytes())
    own = ctx is None
    if own:
        ctx = Context(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    st = torch.cuda.current_stream(dev).cuda_stream
    d_in = torch.from_numpy(np.tile(data, copies)).to(dev)
    offs = np.arange(copies + 1, dtype=np.uint64) * np.uint64(buf_size)
    cap = enc_bound(buf_size)
    cap_offs = np.arange(copies + 1, dtype=np.uint64) * np.uint64(cap)
    d_comp = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_pack = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_dec = torch.empty(buf_size * copies, dtype=torch.uint8, device=dev)
    sizes = np.full(copies, buf_size, dtype=np.int64)
    tot_bench = tot_enc = tot_dec = tot_comp = 0
    comp_size = None
    try:
        for _ in range(num_iterations):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
            encode_ms = int((time.perf_counter() - t0) * 1000)
            if len(set(int(x) for x in lens)) != 1:
                raise RuntimeError("Encoding error")   # identical copies must give identical streams
            if comp_size is None:
                comp_size = int(lens[0])
            elif comp_size != int(lens[0]):
                raise RuntimeError("Encoding error")   # LzmaBench.java:372-374
            pk = ctx.pack_dev(d_comp, cap_offs, lens, d_pack, st)
            decode_ms = 0
            for _ in range(2):   # LzmaBench.java:380-393
                torch.cuda.synchronize(dev)
                t1 = time.perf_counter()
                dlens, status = ctx.decode_batch_dev(props, d_pack, pk, sizes, d_dec, offs, st)
                decode_ms = int((time.perf_counter() - t1) * 1000)
                if (status != 0).any():
                    raise RuntimeError("Decoding Error")
                host = d_dec.cpu().numpy()
                for c in range(copies):
                    if zlib.crc32(host[c * buf_size:(c + 1) * buf_size].tobytes()) != crc:
                        raise RuntimeError("CRC Error")
            bench_size = buf_size * copies
            out.write(results(dictionary_size, encode_ms, bench_size, False, 0) + "     " +
                      results(dictionary_size, decode_ms, buf_size * copies, True, comp_size * copies) + "\n")
            tot_bench += bench_size
            tot_enc += encode_ms
            tot_dec += decode_ms
            tot_comp += comp_size * copies
        out.write("---------------------------------------------------\n")
        out.write(results(dictionary_size, tot_enc, tot_bench, False, 0) + "     " +
                  results(dictionary_size, tot_dec, buf_size * copies * num_iterations, True, tot_comp) +
                  "    Average\n")
    finally:
        if own:
            ctx.close()
    return 0


def main(argv=None):
    """`python -m lzma_amd.lzmabench [passes] [-dN] [-cK]` like `LzmaAlone b [passes] -dN`
    (LzmaAlone.java:170-178: dictionary 2^21 by default); -cK runs K copies per pass."""
    argv = sys.argv[1:] if argv is None else argv
    passes, dict_log, copies = 10, 21, 1
    for a in argv:
        if a.startswith("-d"):
            dict_log = int(a[2:])
        elif a.startswith("-c"):
            copies = int(a[2:])
        else:
            passes = int(a)
    return lzma_benchmark(passes, 1 << dict_log, copies=copies)


if __name__ == "__main__":
    sys.exit(main())
