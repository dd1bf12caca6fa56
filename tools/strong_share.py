"""Strong-scaling projection from one GPU (north_star: one 1 GB buffer at 1/2/4/8 GPUs).

`bench.py --strong` deals the buffer's streams round-robin, rank r taking
{i : i mod G = r} (lzma_amd.dist.rank_streams). Each rank's work is then an
independent batch of n/G streams, so one rank's step time on one GPU is the
G-GPU job's step time up to the max over ranks (the shares differ only in
which bytes they hold). This script times rank 0's share for each G on the
local GPU: encode + pack + decode of the share, device-resident, 1 warm-up
and --steps timed steps, and prints one JSON line per G with the projected
job MB/s = buffer bytes / share step time. It is a PROJECTION: the 8-GPU run
itself is the driver's to measure.

usage: python tools/strong_share.py [--size BYTES] [--chunk BYTES] [--gpus 1,2,4,8] [--steps 2]
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
from lzma_amd import dist as lzdist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1 << 30)
    ap.add_argument("--chunk", type=int, default=256 << 10)
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--dict-log", type=int, default=26)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    p = lzma_amd.make_params(dict_size=1 << args.dict_log, fb=32, mf=1, lc=3, lp=0, pb=2)
    props = lzma_amd.write_props(p)
    full = lzma_amd.bench_generate(args.size)
    n_all = (args.size + args.chunk - 1) // args.chunk
    all_offs = np.minimum(np.arange(n_all + 1, dtype=np.uint64) * np.uint64(args.chunk), np.uint64(args.size))
    ctx, ctx_dec = lzma_amd.Context(0), lzma_amd.Context(0)
    ctx.set_batch_bytes(1 << 30)
    for g in [int(x) for x in args.gpus.split(",")]:
        mine = lzdist.rank_streams(n_all, 0, g)
        host = np.concatenate([full[int(all_offs[i]):int(all_offs[i + 1])] for i in mine])
        lens_in = (all_offs[1:] - all_offs[:-1])[mine]
        n = int(mine.size)
        offs = np.zeros(n + 1, dtype=np.uint64)
        offs[1:] = np.cumsum(lens_in)
        caps = np.array([lzma_amd.enc_bound(int(x)) for x in lens_in], dtype=np.uint64)
        cap_offs = np.zeros(n + 1, dtype=np.uint64)
        cap_offs[1:] = np.cumsum(caps)
        d_in = torch.from_numpy(host).to(dev)
        d_comp = torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=dev)
        d_pack = torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=dev)
        d_dec = torch.empty(host.size + 1, dtype=torch.uint8, device=dev)

        def step():
            lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
            pk = ctx.pack_dev(d_comp, cap_offs, lens, d_pack, st)
            dl, ds = ctx_dec.decode_batch_dev(props, d_pack, pk, lens_in.astype(np.int64), d_dec, offs, st)
            return lens, dl, ds

        step()
        for c in (ctx, ctx_dec):
            c.set_timing(True)
            c.reset_timings()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            lens, dl, ds = step()
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / args.steps
        tm = ctx.timings()
        tm.update(ctx_dec.timings())
        for c in (ctx, ctx_dec):
            c.set_timing(False)
        ok = bool((ds == 0).all()) and bool((dl == lens_in).all()) and bool(torch.equal(d_dec[:host.size], d_in))
        print(json.dumps({
            "row": "strong_share", "gpus": g, "rank": 0, "streams": n, "bytes": int(host.size),
            "step_ms": dt * 1e3, "projected_job_MBps": args.size / dt / 1e6,
            "kernels_ms_per_step": {k: v[0] / args.steps for k, v in sorted(tm.items())},
            "ratio": float(np.sum(lens)) / host.size, "roundtrip_ok": ok,
            "label": "projection from one GPU (rank 0's share of --strong); unmeasured on %d GPUs" % g}), flush=True)
        del d_in, d_comp, d_pack, d_dec
    ctx.close()
    ctx_dec.close()


if __name__ == "__main__":
    main()
