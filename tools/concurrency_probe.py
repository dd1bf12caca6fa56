"""Encode beside a running decode, on two HIP streams (no fence): does the
match finder make progress while the batch decoder runs, and are both results
right? Bench workload (1 GiB, 4096 x 256 KiB, dict 2^26 L5). Prints progress
to stderr and one JSON line: the sequential encode / decode times, the
concurrent wall time, and whether the concurrent decode round-tripped and the
concurrent encode's lengths equal the sequential ones.

usage: LZMA_AMD_LIB=... python tools/concurrency_probe.py [--size BYTES]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402


def log(msg):
    print("[probe %.3f] %s" % (time.perf_counter(), msg), file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
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
    d_comp2 = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_pack = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    d_dec = torch.empty(args.size, dtype=torch.uint8, device=dev)
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32)
    props = lzma_amd.write_props(p)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    ctx, cdec = lzma_amd.Context(0), lzma_amd.Context(0)
    ctx.set_batch_bytes(1 << 30)
    sizes = np.full(n, chunk, dtype=np.int64)
    torch.cuda.synchronize()
    res = {"lib": lzma_amd.LIB_PATH}
    t0 = time.perf_counter()
    lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, sa.cuda_stream)
    res["enc_alone_ms"] = (time.perf_counter() - t0) * 1e3
    pk = ctx.pack_dev(d_comp, cap_offs, lens, d_pack, sa.cuda_stream)
    log("sequential encode done")
    t0 = time.perf_counter()
    cdec.decode_batch_dev(props, d_pack, pk, sizes, d_dec, offs, sb.cuda_stream)
    res["dec_alone_ms"] = (time.perf_counter() - t0) * 1e3
    log("sequential decode done")
    d_dec.zero_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cdec.decode_batch_dev_async(props, d_pack, pk, sizes, d_dec, offs, sb.cuda_stream)
    done = {}

    def waiter():
        dl, ds = cdec.decode_batch_dev_wait()
        done["dec_ms"] = (time.perf_counter() - t0) * 1e3
        done["dec_ok"] = bool((ds == 0).all()) and bool((dl == sizes).all())
        log("concurrent decode done")

    th = threading.Thread(target=waiter)
    th.start()
    lens2 = ctx.encode_batch_dev(d_in, offs, p, d_comp2, cap_offs, sa.cuda_stream)
    res["enc_concurrent_ms"] = (time.perf_counter() - t0) * 1e3
    log("concurrent encode done")
    th.join()
    torch.cuda.synchronize()
    res["wall_concurrent_ms"] = (time.perf_counter() - t0) * 1e3
    res["dec_concurrent_ms"] = done.get("dec_ms")
    res["dec_ok"] = done.get("dec_ok", False) and bool(torch.equal(d_dec, d_in))
    res["enc_ok"] = bool(np.array_equal(lens, lens2))
    if res["enc_ok"]:   # every stream of the concurrent encode byte-equal to the sequential one
        d_pack2 = torch.empty_like(d_pack)
        pk2 = ctx.pack_dev(d_comp2, cap_offs, lens2, d_pack2, sa.cuda_stream)
        torch.cuda.synchronize()
        res["enc_bytes_equal"] = bool(np.array_equal(pk, pk2)) and bool(torch.equal(d_pack[:int(pk[-1])], d_pack2[:int(pk2[-1])]))
        # and a sample of them equal to the oracle's Encoder.Code bytes
        sys.path.insert(0, os.path.join(REPO, "tests"))
        import oracle_ffi as orc
        idx = np.linspace(0, n - 1, 16).astype(int)
        hp = d_pack2[:int(pk2[-1])].cpu().numpy()
        ref = orc.encode_many([host[int(offs[i]):int(offs[i + 1])].tobytes() for i in idx],
                              orc.params(1 << 26, 32, 1, 3, 0, 2, 0), threads=orc.cpu_threads())
        res["oracle_sample_equal"] = all(hp[int(pk2[i]):int(pk2[i + 1])].tobytes() == r for i, r in zip(idx, ref))
    res["timings"] = {k: round(v[0], 1) for k, v in ctx.timings().items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
