"""Encoder throughput vs. number of concurrent streams (device-resident).

usage: python tools/enc_scaling.py [chunk_bytes] [counts_csv] [bench|text] [dict_log]
With LZMA_AMD_LIB=lzma-java_amd/build/prof/liblzma_mi355x.so the library
prints the per-phase cycle profile of each pass to stderr.
"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402


def main():
    chunk = int(sys.argv[1]) if len(sys.argv) > 1 else 256 << 10
    counts = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,64,256,1024").split(",")]
    kind = sys.argv[3] if len(sys.argv) > 3 else "bench"
    dict_log = int(sys.argv[4]) if len(sys.argv) > 4 else (28 if kind == "text" else 26)
    dev = torch.device("cuda", 0)
    total = chunk * max(counts)
    host = lzma_amd.generate(kind, total)
    d_in = torch.from_numpy(host).to(dev)
    p = lzma_amd.make_params(dict_size=1 << dict_log, fb=32, mf=1, lc=3, lp=0, pb=2)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(max(total, 1 << 20))
    st = torch.cuda.current_stream(dev).cuda_stream
    for n in counts:
        offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk)
        caps = np.array([lzma_amd.enc_bound(chunk)] * n, dtype=np.uint64)
        cap_offs = np.zeros(n + 1, dtype=np.uint64)
        cap_offs[1:] = np.cumsum(caps)
        d_out = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
        ctx.set_timing(True)
        ctx.reset_timings()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lens = ctx.encode_batch_dev(d_in, offs, p, d_out, cap_offs, st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tm = ctx.timings()
        parse = tm.get("enc_parse", (0.0, 0))[0]
        print("streams=%5d bytes=%10d wall=%.3fs enc_parse=%.1fms -> %.2f MB/s (parse-only %.2f MB/s) ratio=%.4f"
              % (n, n * chunk, dt, parse, n * chunk / dt / 1e6, n * chunk / max(parse, 1e-6) / 1e3,
                 float(np.sum(lens)) / (n * chunk)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
