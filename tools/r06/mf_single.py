"""The match finder's kernels on ONE long stream (config 4's shape): lzma_enc_session_begin
runs the whole-stream match finder; HIP-event times per kernel name.
usage: python tools/r06/mf_single.py [MiB]"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n = mib << 20
    data = lzma_amd.bench_generate(n)
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(data).to(dev)
    cap = lzma_amd.enc_bound(n)
    d_out = torch.empty(cap + 1, dtype=torch.uint8, device=dev)
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32, mf=1)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(max(1 << 30, n))
    ctx.set_timing(True)
    torch.cuda.synchronize(dev)
    t0 = time.time()
    s = ctx.session(d_in, n, p, d_out, cap, torch.cuda.current_stream(dev).cuda_stream)
    t1 = time.time()
    s.step(1 << 20)
    t2 = time.time()
    tm = ctx.timings()
    s.close()
    ctx.close()
    print(json.dumps({"mib": mib, "begin_s": t1 - t0, "first_MiB_step_s": t2 - t1,
                      "kernels_ms": {k: round(v[0], 1) for k, v in sorted(tm.items(), key=lambda kv: -kv[1][0])}}))


if __name__ == "__main__":
    main()
