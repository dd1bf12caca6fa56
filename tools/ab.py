"""A/B timing of one library build on the bench workload (1 GiB LzmaBench
data, 4096 x 256 KiB streams, dict 2^26 L5): encode + pack + decode, one
warm-up and --reps timed repetitions, per-kernel HIP-event times, the round
trip and an oracle parity sample. One JSON line. The library is the one
LZMA_AMD_LIB names (default: the product build).

usage: LZMA_AMD_LIB=build/x/liblzma_mi355x.so python tools/ab.py [--reps 2] [--parity 8]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--parity", type=int, default=8)
    ap.add_argument("--size", type=int, default=1 << 30)
    ap.add_argument("--chunk", type=int, default=256 << 10)
    ap.add_argument("--data", choices=["bench", "text"], default="bench")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    host = lzma_amd.generate(args.data, args.size)
    dict_log = 28 if args.data == "text" else 26
    n = args.size // args.chunk
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(args.chunk)
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum([lzma_amd.enc_bound(args.chunk)] * n)
    d_in = torch.from_numpy(host).to(dev)
    d_comp = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_pack = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_dec = torch.empty(args.size, dtype=torch.uint8, device=dev)
    p = lzma_amd.make_params(dict_size=1 << dict_log, fb=32, mf=1, lc=3, lp=0, pb=2)
    props = lzma_amd.write_props(p)
    ctx, cdec = lzma_amd.Context(0), lzma_amd.Context(0)
    ctx.set_batch_bytes(1 << 30)
    sizes = np.full(n, args.chunk, dtype=np.int64)
    res = {"lib": os.environ.get("LZMA_AMD_LIB", "product"), "data": args.data}
    walls = []
    for rep in range(args.reps + 1):
        if rep == 1:
            for c in (ctx, cdec):
                c.set_timing(True)
                c.reset_timings()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
        pk = ctx.pack_dev(d_comp, cap_offs, lens, d_pack, st)
        t1 = time.perf_counter()
        dl, ds = cdec.decode_batch_dev(props, d_pack, pk, sizes, d_dec, offs, st)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        if rep:
            walls.append((t1 - t0, t2 - t1))
    tm = ctx.timings()
    tm.update(cdec.timings())
    ok = bool((ds == 0).all()) and bool(torch.equal(d_dec, d_in))
    par = None
    if args.parity:
        import oracle_ffi as orc
        idx = np.linspace(0, n - 1, args.parity).astype(int)
        hp = d_pack[:int(pk[-1])].cpu().numpy()
        ref = orc.encode_many([host[int(offs[i]):int(offs[i + 1])].tobytes() for i in idx],
                              orc.params(1 << dict_log, 32, 1, 3, 0, 2, 0))
        par = all(hp[int(pk[i]):int(pk[i + 1])].tobytes() == r for i, r in zip(idx, ref))
    enc_s = min(w[0] for w in walls)
    dec_s = min(w[1] for w in walls)
    res.update(enc_s=enc_s, dec_s=dec_s, MBps=args.size / (enc_s + dec_s) / 1e6,
               kernels_ms={k: round(v[0] / args.reps, 2) for k, v in tm.items()},
               roundtrip=ok, parity=par, ratio=float(lens.sum()) / args.size)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
