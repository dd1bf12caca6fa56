"""Staged GPU probe: encode increasingly large inputs, compare with the oracle,
print timing per stage immediately (debugging aid)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lzma-java_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import lzma_amd  # noqa: E402
import oracle_ffi as orc  # noqa: E402

sizes = [int(x) for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else [16, 300, 4096, 65536]
fb = int(sys.argv[2]) if len(sys.argv) > 2 else 32
ctx = lzma_amd.Context(0)
p = lzma_amd.make_params(dict_size=1 << 23, fb=fb)
op = orc.params(p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos)
for n in sizes:
    data = lzma_amd.bench_generate(n).tobytes()
    t = time.time()
    out = ctx.encode_batch([data], p)[0]
    dt = time.time() - t
    ok = out == orc.encode(data, op)
    print("n=%d fb=%d gpu %.3fs ok=%s len=%d" % (n, fb, dt, ok, len(out)), flush=True)
