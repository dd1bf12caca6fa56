"""Benchmark: compress+decompress MB/s on 1 GiB of synthetic low-entropy data per GPU.

Workload (BASELINE.json metric / configs 2 and 4): the reference's own
LzmaBench generator (LzmaBench.java:15-127), 1 GiB per rank, split into
independent LZMA streams of --chunk bytes (default 256 KiB), each encoded
exactly as Encoder.Code would with the level-5 mapping:
dict 2^26, fb 32, BT4, lc3 lp0 pb2. A step = encode every stream (GPU),
pack the outputs into one contiguous container (GPU), decode every stream
(GPU). Inputs are resident in HBM before the timed region. Scaling is weak:
each rank processes its own 1 GiB with no data-path collective; with N > 1
ranks the step ends with the one exchange SURVEY.md 8(e) prescribes -- rank 0
gathers every rank's packed streams over RCCL (lzma_amd.dist.gather_streams).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402
from lzma_amd import dist as lzdist  # noqa: E402

HBM_PEAK = 8.0e12   # MI355X HBM3E, MI355X_MICROARCH.md chip-level parameters


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size", type=int, default=1 << 30, help="uncompressed bytes per GPU")
    ap.add_argument("--chunk", type=int, default=256 << 10, help="bytes per independent stream")
    ap.add_argument("--batch-bytes", type=int, default=1 << 30,
                    help="input bytes per device pass (1 GiB: all streams of a GPU in one encoder launch)")
    ap.add_argument("--cpu-sample", type=int, default=32 << 20, help="bytes for the CPU baseline (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16, help="threads for the multi-core CPU baseline")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--overlap", action="store_true",
                    help="pipeline the steps: the decode of step k runs on its own HIP stream and context while "
                         "step k+1 encodes (default: each step's encode and decode run back to back)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as td
        torch.cuda.set_device(local)
        td.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    # ---- synthetic data (host gen, then H2D; outside the timed region)
    size = args.size
    host = lzma_amd.bench_generate(size)
    if rank:   # distinct streams per rank: the generator output rotated by a rank-dependent odd offset
        host = np.roll(host, -(rank * 262147) % size)
    d_in = torch.from_numpy(host).to(dev)
    n = (size + args.chunk - 1) // args.chunk
    offs = np.minimum(np.arange(n + 1, dtype=np.uint64) * np.uint64(args.chunk), np.uint64(size))
    caps = np.array([lzma_amd.enc_bound(int(offs[i + 1] - offs[i])) for i in range(n)], dtype=np.uint64)
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum(caps)
    d_comp = torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev)
    # two packed buffers: step k's decode reads one while step k+1 packs into the other
    d_packs = [torch.empty(int(cap_offs[-1]), dtype=torch.uint8, device=dev) for _ in range(2)]
    d_dec = torch.empty(size, dtype=torch.uint8, device=dev)
    out_sizes = (offs[1:] - offs[:-1]).astype(np.int64)

    p = lzma_amd.make_params(dict_size=1 << 26, fb=32, mf=1, lc=3, lp=0, pb=2)
    props = lzma_amd.write_props(p)
    ctx = lzma_amd.Context(dev.index)
    ctx.set_batch_bytes(args.batch_bytes)
    st = torch.cuda.current_stream(dev).cuda_stream
    # the decoder gets its own context (its own device workspace) and HIP stream; with
    # --overlap a step's decode runs while the next step encodes (measured: +3 %, the
    # decoder and the match-finder sorts slow each other down). Every step still
    # encodes and decodes all its bytes.
    ctx_dec = lzma_amd.Context(dev.index)
    dec_stream = torch.cuda.Stream(dev)
    st_dec = dec_stream.cuda_stream

    state = {}
    pending = []

    def decode(buf, pk):
        try:
            t1 = time.perf_counter()
            dlens, dstat = ctx_dec.decode_batch_dev(props, buf, pk, out_sizes, d_dec, offs, st_dec)
            state["dstat"], state["dlens"] = dstat, dlens
            state["t_dec"] = state.get("t_dec", 0.0) + (time.perf_counter() - t1)
        except BaseException as e:   # re-raised by join() in the main thread
            state["dec_error"] = e

    def join():
        while pending:
            pending.pop().join()
        if "dec_error" in state:
            raise state.pop("dec_error")

    def step(k):
        t0 = time.perf_counter()
        lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
        buf = d_packs[k % 2]
        pk = ctx.pack_dev(d_comp, cap_offs, lens, buf, st)   # synchronous: buf is complete
        if dist:   # the single data exchange: rank 0 collects every rank's packed streams
            g, _, _ = lzdist.gather_streams(buf, lens, dst=0)
            state["gathered"] = 0 if g is None else int(g.numel())
        state["lens"] = lens
        state["t_enc"] = state.get("t_enc", 0.0) + (time.perf_counter() - t0)
        join()                           # one decode in flight at a time (d_dec is shared)
        if not args.overlap:
            decode(buf, pk)
        else:
            th = threading.Thread(target=decode, args=(buf, pk))
            th.start()
            pending.append(th)

    for k in range(args.warmup):
        step(k)
    join()

    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    for c in (ctx, ctx_dec):
        c.set_timing(True)
        c.reset_timings()
    state["t_enc"] = state["t_dec"] = 0.0
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k)
    join()
    barrier()
    elapsed = time.perf_counter() - t0
    timings = ctx.timings()
    timings.update(ctx_dec.timings())
    for c in (ctx, ctx_dec):
        c.set_timing(False)

    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())

    comp_bytes = int(np.sum(state["lens"]))
    ok = bool((state["dstat"] == 0).all()) and bool((state["dlens"] == out_sizes).all())
    if not args.no_verify:
        ok = ok and bool(torch.equal(d_dec, d_in))
    if dist:
        flag = torch.tensor([1 if ok else 0], device=dev)
        torch.distributed.all_reduce(flag, op=torch.distributed.ReduceOp.MIN)
        ok = bool(flag.item())

    total_bytes = size * world * args.steps
    value = total_bytes / elapsed / 1e6

    # ---- roofline for the dominant kernel (HIP events on the launch stream)
    dom = max(timings.items(), key=lambda kv: kv[1][0]) if timings else ("none", (0.0, 1))
    dname, (dms, dlaunch) = dom
    avg_s = dms / 1e3 / max(dlaunch, 1)
    per_step_launches = max(dlaunch // max(args.steps, 1), 1)
    if dname.startswith("dec"):
        alg = (comp_bytes + size) / per_step_launches    # N_comp + N_out per launch
    else:
        alg = (size + comp_bytes) / per_step_launches    # N_in + N_out per launch
    achieved = alg / avg_s if avg_s > 0 else 0.0
    traffic, traffic_src = pmc_traffic(dname, args.size, args.chunk)
    roofline = {"bound": "hbm", "kernel": dname, "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                "unit": "GB/s", "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_source": traffic_src,
                "avg_launch_ms": avg_s * 1e3, "launches_per_step": per_step_launches,
                "alg_bytes_per_launch": alg}

    cpu = None
    if rank == 0 and args.cpu_sample > 0 and world == 1:
        cpu = cpu_baseline(host, args.chunk, args.cpu_sample, p, args.cpu_threads)

    if rank == 0:
        res = {
            "metric": "compress+decompress MB/s on 1 GB synthetic; bit-exact .lzma vs Java ref",
            "value": value, "unit": "MB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (LzmaBench CBenchRandomGenerator)",
            "config": {"workload": "LzmaBench generator %d MiB per GPU as %d independent streams of %d KiB; "
                                   "dict 2^26 fb32 bt4 lc3 lp0 pb2 (level-5 mapping); encode+pack+decode"
                                   % (size >> 20, n, args.chunk >> 10),
                       "bytes_per_gpu": size, "chunk": args.chunk, "streams_per_gpu": n,
                       "parallelism": "independent streams, %d rank(s)" % world},
            "compress_MBps": size * world * args.steps / max(state["t_enc"], 1e-9) / 1e6,
            "decompress_MBps": size * world * args.steps / max(state["t_dec"], 1e-9) / 1e6,
            "schedule": "sequential" if not args.overlap else
                        "pipelined: step k's decode (own context + HIP stream) overlaps step k+1's encode; "
                        "compress/decompress MB/s are each phase's own wall time",
            "ratio": comp_bytes / size, "verified": ok,
            "gathered_bytes_rank0": state.get("gathered"),
            "kernels_ms": {k: {"total_ms": v[0], "launches": v[1]} for k, v in timings.items()},
            "roofline": roofline, "cpu_baseline": cpu,
        }
        print(json.dumps(res), flush=True)
    ctx.close()
    ctx_dec.close()
    if dist:
        torch.distributed.destroy_process_group()
    if not ok:
        sys.exit(1)


# HIP-event timing label -> rocprofv3 kernel-name prefix
_KERNEL_OF = {"enc_parse": "enc_kernel", "dec_stream": "dec_kernel", "mf_walk": "mf_walk_kernel"}


def pmc_traffic(label, size, chunk):
    """HBM bytes per launch of the dominant kernel from the committed PMC
    summary (profiles/traffic.json, written by tools/profile_round.sh from
    separate FETCH_SIZE / WRITE_SIZE passes over this same workload), or None
    when that summary is absent or was taken on another workload."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        t = json.load(f)
    meta = t.get("_workload", {})
    if meta.get("bytes_per_gpu") != size or meta.get("chunk") != chunk:
        return None, None
    prefix = _KERNEL_OF.get(label, label)
    for k, v in t.items():
        if k.startswith(prefix) and isinstance(v, dict) and "traffic_bytes_per_launch" in v:
            return v["traffic_bytes_per_launch"], "profiles/traffic.json (%s, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)" % k
    return None, None


def cpu_baseline(host, chunk, sample, p, threads):
    """C restatement of the reference (oracle/) on a bounded sample of the same
    chunks: encode + decode, MB/s of uncompressed bytes. Timed with 1 thread
    (the reference is single-threaded) and with `threads` threads, one chunk
    per task (ctypes releases the GIL inside the C calls); `value` is the
    multi-thread figure."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as orc
    from concurrent.futures import ThreadPoolExecutor
    op = orc.params(p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos)
    props = orc.props(op)
    sample = min(sample, host.size)
    chunks = [host[i:min(i + chunk, sample)].tobytes() for i in range(0, sample, chunk)]

    def enc(c):
        return orc.encode(c, op)

    def dec(args):
        c, e = args
        rc, d = orc.decode(e, props, len(c))
        assert rc == 1 and d == c

    def timed(nthreads):
        with ThreadPoolExecutor(max_workers=nthreads) as ex:
            t0 = time.perf_counter()
            encs = list(ex.map(enc, chunks))
            t1 = time.perf_counter()
            list(ex.map(dec, zip(chunks, encs)))
            t2 = time.perf_counter()
        return sample / (t2 - t0) / 1e6, sample / (t1 - t0) / 1e6, sample / (t2 - t1) / 1e6

    one = timed(1)
    threads = max(1, min(threads, len(chunks)))
    multi = timed(threads) if threads > 1 else one
    return {"value": multi[0], "unit": "MB/s", "cores": threads, "kind": "port",
            "compress_MBps": multi[1], "decompress_MBps": multi[2],
            "single_thread": {"value": one[0], "compress_MBps": one[1], "decompress_MBps": one[2], "cores": 1},
            "sample": "first %d MiB of the same workload (%d streams of %d KiB), oracle/ C restatement of the "
                      "Java reference (no JDK on the box), %d threads; single_thread = 1 thread"
                      % (sample >> 20, len(chunks), chunk >> 10, threads)}


if __name__ == "__main__":
    main()
