"""The single-stream C ABI (lzma_encode / lzma_decode, the JNI shim's calls) repeated on
one context, for a rocprofv3 --hip-trace summary: after the first call the context's
device buffers are reused, so hipMalloc / hipFree must not scale with the call count.

usage: rocprofv3 --hip-trace --stats -d DIR -o run -- python3 tools/c_abi_repeat.py [calls]
"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    L = lzma_amd.lib()
    ctx = lzma_amd.Context(0)
    data = lzma_amd.bench_generate(1 << 16).tobytes()
    p = lzma_amd.make_params(dict_size=1 << 20, fb=32)
    props = (ctypes.c_uint8 * 5)(*lzma_amd.write_props(p))
    cap = lzma_amd.enc_bound(len(data))
    out = ctypes.create_string_buffer(cap)
    dec = ctypes.create_string_buffer(len(data) + 273)
    n_out, n_dec = ctypes.c_uint64(), ctypes.c_uint64()
    first = None
    for i in range(calls):
        rc = L.lzma_encode(ctx.h, ctypes.byref(p), data, len(data), out, cap, ctypes.byref(n_out))
        assert rc == 0, ctx.error()
        enc = out.raw[:n_out.value]
        first = first or enc
        assert enc == first
        rc = L.lzma_decode(ctx.h, props, enc, len(enc), len(data), dec, len(dec), ctypes.byref(n_dec))
        assert rc == 0 and dec.raw[:n_dec.value] == data
    ctx.close()
    print("c_abi_repeat: %d encode+decode calls on one context, %d -> %d bytes" % (calls, len(data), len(first)))


if __name__ == "__main__":
    main()
