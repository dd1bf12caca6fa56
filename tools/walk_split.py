"""Timing experiment: the match-finder walk restricted to chains of length in
[lo, hi] (LZG_WALK_ONLY=lo,hi; the output is then incomplete, so the encode's
status is ignored). Shows how much of mf_walk is the long-chain tail.

usage: LZG_WALK_ONLY=lo,hi python tools/walk_split.py [bench|text] [bytes]
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "text"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 30
    chunk = 256 << 10
    dev = torch.device("cuda", 0)
    host = lzma_amd.generate(kind, size)
    d_in = torch.from_numpy(host).to(dev)
    n = size // chunk
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk)
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum([lzma_amd.enc_bound(chunk)] * n)
    d_out = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    p = lzma_amd.make_params(dict_size=1 << (28 if kind == "text" else 26), fb=32, mf=1, lc=3, lp=0, pb=2)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(max(size, 1 << 20))
    st = torch.cuda.current_stream(dev).cuda_stream
    walks = []
    for rep in range(3):
        ctx.set_timing(True)
        ctx.reset_timings()
        try:
            ctx.encode_batch_dev(d_in, offs, p, d_out, cap_offs, st)
        except Exception as e:   # incomplete match lists may trip the parser's checks
            pass
        torch.cuda.synchronize()
        tm = ctx.timings()
        if rep:
            walks.append(tm.get("mf_walk", (0.0, 0))[0])
    print(json.dumps({"kind": kind, "walk_only": os.environ.get("LZG_WALK_ONLY", "all"), "mf_walk_ms": walks}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
