"""A/B timing of one library build in the few-streams regime (the solo parse kernel):
one long stream and the strong-scaling per-rank shares (512 / 1024 streams of
256 KiB), LzmaBench data, dict 2^26 L5. Per row: encode wall time, the parse
kernel's HIP-event time, cycles per byte of one stream (2.4 GHz), and parity of
the row's first stream against the oracle. One JSON line per row. The library
is the one LZMA_AMD_LIB names (default: the product build).

usage: LZMA_AMD_LIB=... python tools/ab_solo.py [--single BYTES] [--shares 512,1024]
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
sys.path.insert(0, os.path.join(REPO, "tests"))
import lzma_amd  # noqa: E402
import oracle_ffi as orc  # noqa: E402

CLOCK = 2.4e9


def run(ctx, host, n, chunk, p, dev, st, label, parity=True):
    offs = np.minimum(np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk), np.uint64(host.size))
    lens_in = offs[1:] - offs[:-1]
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum([lzma_amd.enc_bound(int(x)) for x in lens_in])
    d_in = torch.from_numpy(host[:int(offs[-1])]).to(dev)
    d_out = torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=dev)
    ctx.set_timing(True)
    ctx.reset_timings()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    lens = ctx.encode_batch_dev(d_in, offs, p, d_out, cap_offs, st)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    tm = ctx.timings()
    ctx.set_timing(False)
    parse_ms = tm.get("enc_parse", (0.0, 0))[0]
    res = {"row": label, "lib": os.environ.get("LZMA_AMD_LIB", "product"), "streams": n, "chunk": chunk,
           "bytes": int(offs[-1]), "wall_s": wall, "parse_ms": parse_ms,
           "MBps": int(offs[-1]) / wall / 1e6,
           "parse_cycles_per_byte_per_stream": parse_ms / 1e3 * CLOCK / max(int(lens_in[0]), 1),
           "ratio": float(np.sum(lens)) / int(offs[-1]),
           "kernels_ms": {k: round(v[0], 2) for k, v in sorted(tm.items())}}
    if parity:
        first = d_out[:int(lens[0])].cpu().numpy().tobytes()
        op = orc.params(p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos)
        res["first_stream_equals_oracle"] = first == orc.encode(host[:int(offs[1])].tobytes(), op)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--single", type=int, default=4 << 20)
    ap.add_argument("--shares", default="512,1024")
    ap.add_argument("--chunk", type=int, default=256 << 10)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32, mf=1, lc=3, lp=0, pb=2)
    shares = [int(x) for x in args.shares.split(",") if x]
    total = max([args.single] + [n * args.chunk for n in shares])
    host = lzma_amd.bench_generate(total)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(1 << 30)
    run(ctx, host, 64, 64 << 10, p, dev, st, "warmup", parity=False)
    if args.single:
        print(json.dumps(run(ctx, host, 1, args.single, p, dev, st, "single")), flush=True)
    for n in shares:
        print(json.dumps(run(ctx, host, n, args.chunk, p, dev, st, "share")), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
