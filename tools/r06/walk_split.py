"""Where the walk's time goes by chain length (experiment build, LZG_WALK_ONLY).

The bench's batch (4096 streams of 256 KiB, level 5) is encoded once in full, then its match
finder is run with the walk restricted to chains of length [lo, hi] (the parse is refused
under LZG_WALK_ONLY, so each restricted call ends after the walk); HIP-event times per kernel.
usage: LZMA_AMD_LIB=lzma-java_amd/build/exp/liblzma_mi355x.so python tools/r06/walk_split.py [text|bench]
       WALK_FULL_ONLY=1 LZMA_AMD_LIB=<any library> python tools/r06/walk_split.py [text|bench]
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "text"
    total, chunk = 1 << 30, 1 << 18
    n = total // chunk
    data = lzma_amd.generate(kind, total)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(data).to(dev)
    offs = np.arange(n + 1, dtype=np.uint64) * chunk
    caps = np.array([lzma_amd.enc_bound(chunk)] * n, dtype=np.uint64)
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum(caps)
    d_comp = torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=dev)
    p = lzma_amd.make_params(dict_size=1 << (28 if kind == "text" else 26), fb=32, mf=1, lc=3, lp=0, pb=2)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(total)
    st = torch.cuda.current_stream(dev).cuda_stream
    out = {"data": kind, "streams": n, "chunk": chunk}
    rows = (("all (full encode)", None), ("all", "0,4294967295"), ("< 256", "0,255"),
            (">= 256", "256,4294967295"), (">= 1024", "1024,4294967295"), ("== 1", "1,1"), (">= 2", "2,4294967295"),
            ("none", "4294967295,4294967295"))
    if os.environ.get("WALK_FULL_ONLY"):   # a product-form library (no LZG_WALK_ONLY): full encodes only
        rows = rows[:1]
    for name, rng in rows:
        for rep in range(2):
            if rng is None:
                os.environ.pop("LZG_WALK_ONLY", None)
            else:
                os.environ["LZG_WALK_ONLY"] = rng
            ctx.set_timing(True)
            ctx.reset_timings()
            try:
                ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
            except Exception as e:  # the refused parse of a walk-only pass
                if rng is None:
                    raise
                assert "LZG_WALK_ONLY" in str(e), e
            torch.cuda.synchronize(dev)
            tm = ctx.timings()
            out.setdefault(name, []).append(round(tm.get("mf_walk", (0.0, 0))[0], 1))
        print(name, out[name], flush=True)
    os.environ.pop("LZG_WALK_ONLY", None)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
