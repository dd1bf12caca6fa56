"""Chunk-size sweep and the per-stream serial-tail ceiling.

For each chunk size: the input (LzmaBench or TEXT generator) split into
independent streams of that size, encoded + packed + decoded on the GPU
(device-resident, one untimed warm-up pass for the first row only), with
MB/s and the compression ratio. The first stream of every row is checked
byte for byte against the oracle, and every stream must decode back.

--single N appends one row for a single stream of N bytes timed end to end:
the serial-tail ceiling (one stream is one wave's serial parse).

Prints one JSON line per row.
usage: python tools/chunk_sweep.py [--data bench|text] [--dict-log 26] [--size BYTES]
                                   [--chunks 262144,1048576,...] [--single BYTES]
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


def run(ctx, ctx_dec, host, chunk, p, dev, st, label):
    size = host.size
    n = (size + chunk - 1) // chunk
    offs = np.minimum(np.arange(n + 1, dtype=np.uint64) * np.uint64(chunk), np.uint64(size))
    lens_in = offs[1:] - offs[:-1]
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum([lzma_amd.enc_bound(int(x)) for x in lens_in])
    d_in = torch.from_numpy(host).to(dev)
    d_comp = torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=dev)
    d_pack = torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=dev)
    d_dec = torch.empty(size + 1, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
    pk = ctx.pack_dev(d_comp, cap_offs, lens, d_pack, st)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    dl, ds = ctx_dec.decode_batch_dev(lzma_amd.write_props(p), d_pack, pk, lens_in.astype(np.int64), d_dec, offs, st)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    ok = bool((ds == 0).all()) and bool((dl == lens_in).all()) and bool(torch.equal(d_dec[:size], d_in))
    first = d_pack[:int(pk[1])].cpu().numpy().tobytes()
    op = orc.params(p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos)
    parity = first == orc.EncoderSession(op).encode(host[:int(offs[1])].tobytes())
    comp = int(lens.sum())
    return {"row": label, "chunk": chunk, "streams": n, "bytes": size, "encode_s": t1 - t0, "decode_s": t2 - t1,
            "compress_MBps": size / (t1 - t0) / 1e6, "decompress_MBps": size / (t2 - t1) / 1e6,
            "compress_decompress_MBps": size / (t2 - t0) / 1e6, "ratio": comp / size,
            "roundtrip_ok": ok, "first_stream_equals_oracle": parity}


def heartbeat(period=30.0):
    """A line on stderr every `period` seconds, so a long single-stream run is
    visibly alive (a GPU job that prints nothing for minutes is taken as hung)."""
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(period)
            print("[chunk_sweep] running %.0f s" % (time.time() - t0), file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", choices=["bench", "text"], default="bench")
    ap.add_argument("--dict-log", type=int, default=None)
    ap.add_argument("--size", type=int, default=1 << 30)
    ap.add_argument("--chunks", default="262144,1048576,4194304,16777216")
    ap.add_argument("--single", type=int, default=0, help="bytes of one stream timed end to end (0 = skip)")
    args = ap.parse_args()
    dict_log = args.dict_log if args.dict_log is not None else (28 if args.data == "text" else 26)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream(dev).cuda_stream
    p = lzma_amd.make_params(dict_size=1 << dict_log, fb=32, mf=1, lc=3, lp=0, pb=2)
    ctx, ctx_dec = lzma_amd.Context(0), lzma_amd.Context(0)
    ctx.set_batch_bytes(1 << 30)
    host = lzma_amd.generate(args.data, args.size)
    warm = host[:64 << 20]
    run(ctx, ctx_dec, warm, 256 << 10, p, dev, st, "warmup")
    for c in [int(x) for x in args.chunks.split(",") if x]:
        r = run(ctx, ctx_dec, host, c, p, dev, st, "sweep")
        r.update(data=args.data, dict_log=dict_log)
        print(json.dumps(r), flush=True)
    if args.single:
        r = run(ctx, ctx_dec, host[:args.single], args.single, p, dev, st, "single_stream")
        r.update(data=args.data, dict_log=dict_log)
        print(json.dumps(r), flush=True)
    ctx.close()
    ctx_dec.close()


if __name__ == "__main__":
    main()
