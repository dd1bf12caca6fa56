"""Decoder throughput on the bench workload (device-resident): encode once,
then time the batched decoder alone.

usage: python tools/dec_scaling.py [chunk_bytes] [nstreams] [reps]
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
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    dev = torch.device("cuda", 0)
    total = chunk * n
    host = lzma_amd.bench_generate(total)
    d_in = torch.from_numpy(host).to(dev)
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32, mf=1, lc=3, lp=0, pb=2)
    props = lzma_amd.write_props(p)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(total)
    st = torch.cuda.current_stream(dev).cuda_stream
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk)
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum([lzma_amd.enc_bound(chunk)] * n)
    d_comp = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_pack = torch.empty_like(d_comp)
    d_dec = torch.empty(total, dtype=torch.uint8, device=dev)
    lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
    pk = ctx.pack_dev(d_comp, cap_offs, lens, d_pack, st)
    sizes = (offs[1:] - offs[:-1]).astype(np.int64)
    for r in range(reps):
        ctx.set_timing(True)
        ctx.reset_timings()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dl, ds = ctx.decode_batch_dev(props, d_pack, pk, sizes, d_dec, offs, st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        ms = ctx.timings().get("dec_stream", (0.0, 0))[0]
        ok = bool((ds == 0).all()) and bool(torch.equal(d_dec, d_in))
        print("rep %d: streams=%d dec_stream=%.1f ms wall=%.3f s -> %.0f MB/s ok=%s"
              % (r, n, ms, dt, total / max(ms, 1e-6) / 1e3, ok), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
