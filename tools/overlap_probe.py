"""Concurrency probe (experiment build, `make -C lzma-java_amd exp`): does a batch's walk
hide under another batch's parse? Context A parses a staged bench batch (PROBE_MIB, default 512 MiB, of
256 KiB) on one HIP stream while context B walks its own staged batch on another
(LZG_PROBE_WALK_ONLY: B's parse_async runs the walk only). Prints A's parse time alone
and beside B's walk, and B's walk time, as one JSON line.

usage: LZMA_AMD_LIB=lzma-java_amd/build/exp/liblzma_mi355x.so python tools/overlap_probe.py
"""
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
    size, chunk = int(os.environ.get("PROBE_MIB", "512")) << 20, 256 << 10   # two arenas: 1 GiB each does not fit
    n = size // chunk
    torch.cuda.set_device(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    host = lzma_amd.generate("bench", size)
    d_in = torch.from_numpy(host).cuda()
    offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk)
    caps = np.zeros(n + 1, dtype=np.uint64)
    caps[1:] = np.cumsum([lzma_amd.enc_bound(chunk)] * n)
    outs = [torch.empty(int(caps[-1]), dtype=torch.uint8, device="cuda") for _ in range(2)]
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32)
    A, B, dummy = lzma_amd.Context(0), lzma_amd.Context(0), lzma_amd.Context(0)
    for c in (A, B):
        c.set_batch_bytes(size)
    B.set_parse_fence(dummy)   # B's staging enqueues no walk: its parse_async does
    res = {"alone_ms": [], "beside_ms": [], "walk_b_ms": [], "walk_b_alone_ms": []}

    def parse_ms(c):
        t = c.timings()
        return t["enc_parse"][0] / max(t["enc_parse"][1], 1)

    for rep in range(3):
        for beside in (False, True):
            for c in (A, B):
                c.set_timing(True)
                c.reset_timings()
            A.encode_stage_dev(d_in, offs, p, outs[0], caps, s1.cuda_stream)
            B.encode_stage_dev(d_in, offs, p, outs[1], caps, s2.cuda_stream)
            torch.cuda.synchronize()
            A.encode_parse_dev_async(s1.cuda_stream)   # A's walk ran in its staging: the parse starts now
            os.environ["LZG_PROBE_WALK_ONLY"] = "1"
            if beside:
                B.encode_parse_dev_async(s2.cuda_stream)   # B's walk beside A's parse (the host waits for it)
            os.environ.pop("LZG_PROBE_WALK_ONLY")
            A.encode_parse_dev_wait()
            torch.cuda.synchronize()
            if not beside:
                os.environ["LZG_PROBE_WALK_ONLY"] = "1"
                B.encode_parse_dev_async(s2.cuda_stream)   # B's walk alone
                os.environ.pop("LZG_PROBE_WALK_ONLY")
                torch.cuda.synchronize()
            res["beside_ms" if beside else "alone_ms"].append(parse_ms(A))
            tb = B.timings()["mf_walk"]
            res["walk_b_ms" if beside else "walk_b_alone_ms"].append(tb[0] / max(tb[1], 1))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
