"""Do two HIP streams run concurrently here? A batch decode (4096 x 256 KiB
streams of the bench workload) runs asynchronously on stream B; while it runs,
small probes are issued on stream A and timed from the host: a torch kernel,
a 1 GiB device-to-device copy and a pinned host-to-device copy. With working
concurrency each probe ends long before the decode does.

usage: python tools/stream_probe.py [--prio]   (--prio: A high priority, B low)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prio", action="store_true")
    ap.add_argument("--size", type=int, default=1 << 30)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    chunk = 256 << 10
    host = lzma_amd.bench_generate(args.size)
    n = args.size // chunk
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk)
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum([lzma_amd.enc_bound(chunk)] * n)
    d_in = torch.from_numpy(host).to(dev)
    d_comp = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_pack = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_dec = torch.empty(args.size, dtype=torch.uint8, device=dev)
    d_cpy = torch.empty(args.size, dtype=torch.uint8, device=dev)
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32)
    props = lzma_amd.write_props(p)
    sa = torch.cuda.Stream(dev, priority=-1 if args.prio else 0)
    sb = torch.cuda.Stream(dev, priority=0)
    ctx, cdec = lzma_amd.Context(0), lzma_amd.Context(0)
    ctx.set_batch_bytes(1 << 30)
    torch.cuda.synchronize()
    lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, sa.cuda_stream)
    pk = ctx.pack_dev(d_comp, cap_offs, lens, d_pack, sa.cuda_stream)
    sizes = np.full(n, chunk, dtype=np.int64)
    small = torch.zeros(1024, device=dev)
    pin = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
    res = {"prio": args.prio, "streams": [sa.cuda_stream, sb.cuda_stream]}
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cdec.decode_batch_dev(props, d_pack, pk, sizes, d_dec, offs, sb.cuda_stream)
        res["decode_alone_ms"] = (time.perf_counter() - t0) * 1e3
    probes = {}
    for name in ("kernel", "d2d_1GiB", "h2d_pinned_1MiB"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cdec.decode_batch_dev_async(props, d_pack, pk, sizes, d_dec, offs, sb.cuda_stream)
        t1 = time.perf_counter()
        with torch.cuda.stream(sa):
            if name == "kernel":
                small.add_(1)
            elif name == "d2d_1GiB":
                d_cpy.copy_(d_in)
            else:
                d_cpy[:pin.numel()].copy_(pin, non_blocking=True)
        sa.synchronize()
        t2 = time.perf_counter()
        cdec.decode_batch_dev_wait()
        t3 = time.perf_counter()
        probes[name] = {"enqueue_ms": (t1 - t0) * 1e3, "probe_done_ms": (t2 - t0) * 1e3, "decode_done_ms": (t3 - t0) * 1e3}
    res["probes"] = probes
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
