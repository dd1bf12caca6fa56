"""Parse time of the one-wave vs two-wave parser (enc.hip W2) on few streams per CU.

usage: LZG_ENC_W2=0|1 python tools/r04/w2_probe.py CHUNK COUNTS_CSV [PARITY]
Encodes COUNT streams of CHUNK bytes of the LzmaBench data (dict 2^26, fb32 bt4 lc3
lp0 pb2) device-resident; prints one JSON line per count: enc_parse ms, parse cycles
per byte of one stream (at 2.4 GHz) and, for PARITY streams spread over the batch,
whether the bytes equal the oracle's (tests/oracle_ffi.py, Encoder.Code restated).
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import lzma_amd  # noqa: E402
import oracle_ffi as orc  # noqa: E402


def main():
    chunk = int(sys.argv[1])
    counts = [int(x) for x in sys.argv[2].split(",")]
    parity = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    dev = torch.device("cuda", 0)
    host = lzma_amd.bench_generate(chunk * max(counts))
    d_in = torch.from_numpy(host).to(dev)
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32, mf=1, lc=3, lp=0, pb=2)
    op = orc.params(1 << 26, 32, 1, 3, 0, 2, 0)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(max(chunk * max(counts), 1 << 20))
    st = torch.cuda.current_stream(dev).cuda_stream
    for n in counts:
        offs = np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk)
        cap_offs = np.zeros(n + 1, dtype=np.uint64)
        cap_offs[1:] = np.cumsum([lzma_amd.enc_bound(chunk)] * n)
        d_out = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
        ctx.set_timing(True)
        ctx.reset_timings()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        lens = ctx.encode_batch_dev(d_in, offs, p, d_out, cap_offs, st)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        parse = ctx.timings().get("enc_parse", (0.0, 0))[0]
        ok = None
        if parity:
            idx = sorted(set(np.linspace(0, n - 1, min(parity, n)).astype(int).tolist()))
            hout = d_out.cpu().numpy()
            ref = orc.encode_many([host[int(offs[i]):int(offs[i + 1])].tobytes() for i in idx], op)
            ok = all(hout[int(cap_offs[i]):int(cap_offs[i]) + int(lens[i])].tobytes() == r for i, r in zip(idx, ref))
        print(json.dumps({"w2": os.environ.get("LZG_ENC_W2", "auto"), "streams": n, "chunk": chunk, "wall_s": dt,
                          "enc_parse_ms": parse, "parse_cycles_per_byte": parse / 1e3 * 2.4e9 / chunk,
                          "parity_ok": ok, "ratio": float(np.sum(lens)) / (n * chunk)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
