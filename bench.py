"""Benchmark: compress+decompress MB/s on 1 GiB of synthetic data per job step.

Workload (BASELINE.json metric; configs 2-4): by default the reference's own
LzmaBench generator (LzmaBench.java:15-127), 1 GiB, split into independent
LZMA streams of --chunk bytes (default 256 KiB), each encoded exactly as
Encoder.Code would with the level-5 mapping: dict 2^26,
fb 32, BT4, lc3 lp0 pb2. `--data text` switches to the TEXT ("enwik9-shaped")
generator at dict 2^28 (config 3). A step = encode every stream (GPU), pack
the outputs into one contiguous buffer (GPU), decode every stream (GPU).
Inputs are resident in HBM before the timed region.

Multi-GPU (north_star's "one 1 GB buffer at 1, 2, 4 and 8
GPUs"): one process per GPU. `--gpus N` without WORLD_SIZE in the environment
starts the N rank processes itself (before any GPU call); under
torch.distributed.run the ranks come from the environment. `value` is STRONG
scaling: one --size buffer whose streams are dealt round-robin, rank r taking
{i : i mod G = r}, value = the buffer's bytes / the max-over-ranks step time.
At N > 1 a second timed pass gives the weak-scaling figure (every rank its own
--size buffer) as the extra key `weak_scaling`. Neither has a data-path
collective; each step ends with the one exchange 8(e) prescribes: rank 0
gathers every rank's packed streams over RCCL, and after the timed loop checks
that the multi-member container holds every stream of the buffer.

Parity: `verified` is true only if every stream decodes back to its input
AND every sampled stream's GPU bytes equal the oracle's (the bit-exact C
restatement of Encoder.Code) -- at N=1 the sample is the cpu_baseline's
(spread over the whole buffer) plus the rest of the buffer, at N>1 each rank
checks its own streams.

`--emulate` (CPU tests only): the same code path with CPU tensors, the gloo
backend and the product kernels compiled for the CPU SIMT emulation
(tests/simt, LZMA_AMD_LIB); it measures nothing and exists so that the
launcher, the round-robin deal and the gather run in the CPU test suite.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402
from lzma_amd import dist as lzdist  # noqa: E402

HBM_PEAK = 8.0e12   # MI355X HBM3E, MI355X_MICROARCH.md chip-level parameters
SIMT_LIB = os.path.join(REPO, "tests", "simt", "build", "so", "libsimt_lzma.so")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size", type=int, default=1 << 30,
                    help="uncompressed bytes of the job's buffer (strong scaling; per GPU in the weak pass)")
    ap.add_argument("--chunk", type=int, default=256 << 10, help="bytes per independent stream")
    ap.add_argument("--data", choices=["bench", "text"], default="bench",
                    help="bench: LzmaBench generator (configs 2/4); text: enwik9-shaped TEXT (config 3)")
    ap.add_argument("--dict-log", type=int, default=None, help="log2 dictionary size (default 26; 28 with --data text)")
    ap.add_argument("--strong", action="store_true", help="(kept for old command lines: strong scaling is the default)")
    ap.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling pass")
    ap.add_argument("--batch-bytes", type=int, default=1 << 30,
                    help="input bytes per device pass (1 GiB: all streams of a GPU in one encoder launch)")
    ap.add_argument("--cpu-sample", type=int, default=128 << 20,
                    help="bytes of the workload the multi-thread CPU baseline encodes+decodes (0 = skip)")
    ap.add_argument("--cpu-single", type=int, default=8 << 20, help="bytes for the 1-thread CPU baseline")
    ap.add_argument("--cpu-threads", default="share,node_share,nproc",
                    help="thread counts the multi-thread CPU baseline is timed at: 'share' = the job's CPU quota "
                         "(cgroup cpu.max, else OMP_NUM_THREADS / affinity), 'node_share' = nproc / 8 (one GPU's "
                         "share of an 8-GPU node), 'nproc' = every visible CPU, or integers")
    ap.add_argument("--single-stream", type=int, default=16 << 20,
                    help="bytes of the one-stream measurement after the timed region (SURVEY 7.3's serial tail, "
                         "config 4's regime): GPU encode/decode of one stream beside the oracle on 1 thread (0 = skip)")
    ap.add_argument("--parity-streams", type=int, default=-1,
                    help="streams each rank checks against the oracle (-1 = every stream; at N=1 the "
                         "cpu_baseline sample's oracle bytes are reused and the rest encoded beside them)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--sequential", action="store_true",
                    help="run each step's encode and decode back to back (default: pipelined, step k's decode on "
                         "its own HIP stream and context beside step k+1's match finder; step k+1's parser starts "
                         "when that decode is done, lzma_ctx_set_parse_fence; see --pipeline)")
    ap.add_argument("--pipeline", choices=["split", "decode"], default="split",
                    help="pipelined schedule: split (default) = the split encode: step k's range coder, pack and "
                         "decode beside step k+1's match finder; at <= 8 streams per CU (no parse fence) two "
                         "batches are staged and step k+1's walk runs beside step k's parser; decode = the "
                         "synchronous encode, step k's pack + decode beside step k+1's match finder. Measured: "
                         "4096 streams 871 vs 884 ms per step, the 8-way share 508 vs 537 ms "
                         "(profiles/r05/pipe_ab.jsonl, strong_share*.jsonl)")
    ap.add_argument("--emulate", action="store_true",
                    help="CPU tests only: CPU tensors, gloo and the SIMT-emulated product kernels (measures nothing)")
    ap.add_argument("--project-share", type=int, default=1,
                    help="PROJECTION (one GPU, no process group): time rank 0's share of the buffer dealt over G "
                         "GPUs; value = the buffer's bytes / that share's step time (the G-GPU run is the driver's)")
    ap.add_argument("--dump-container", default=None,
                    help="rank 0 writes the gathered multi-member container of the strong pass to this path")
    return ap.parse_args()


def spread(n, k):
    """k stream indices spread evenly over n streams (all of them when k >= n)."""
    if k >= n:
        return list(range(n))
    return sorted(set(int(i) for i in np.linspace(0, n - 1, k).round()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`--gpus N` outside torch.distributed.run: start one rank process per GPU with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set (rendezvous on 127.0.0.1), before
    this process makes any GPU call, and exit with the first failing rank's code.
    If a rank fails, the others (which would wait in a collective) are stopped."""
    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code and not rc:
                rc = code
                for q in live:   # the ranks this launcher started, by their own handles
                    q.terminate()
        time.sleep(0.2)
    return rc


class Device:
    """The rank's device: one MI355X (HIP streams from torch), or the CPU under --emulate."""

    def __init__(self, emulate, local):
        self.emulate = emulate
        if emulate:
            self.dev = torch.device("cpu")
            self.index = 0
        else:
            torch.cuda.set_device(local)
            self.dev = torch.device("cuda", local)
            self.index = local

    def sync(self):
        if not self.emulate:
            torch.cuda.synchronize(self.dev)

    def cus(self):
        return 256 if self.emulate else torch.cuda.get_device_properties(self.dev).multi_processor_count

    def new_stream(self):
        # the encoder and decoder run on HIP streams of their own: work on the null stream
        # would wait for every other stream's work
        return 0 if self.emulate else torch.cuda.Stream(self.dev).cuda_stream


def make_input(args, rank, world, strong):
    """The rank's whole buffer: one shared buffer (strong), or its own (weak; rank 0's
    equals the shared one, so at N = 1 both passes are the same workload)."""
    size = args.size
    if args.data == "text":
        return lzma_amd.text_generate(size, 1 if strong else 1 + rank)
    host = lzma_amd.bench_generate(size)
    if rank and not strong:   # distinct streams per rank: the generator output rotated by an odd offset
        host = np.roll(host, -(rank * 262147) % size)
    return host


def run_pass(args, D, p, ctxs, strong, rank, world, dist):
    """Warm-up + timed steps of one scaling mode; returns its measurements."""
    ctx, ctx_dec, st, st_dec = ctxs
    overlap = not args.sequential
    full = make_input(args, rank, world, strong)
    size = full.size
    n_all = (size + args.chunk - 1) // args.chunk
    all_offs = np.minimum(np.arange(n_all + 1, dtype=np.uint64) * np.uint64(args.chunk), np.uint64(size))
    deal = max(world, args.project_share)   # --project-share: rank 0's share of a G-way deal, on one GPU
    mine = lzdist.rank_streams(n_all, rank, deal) if strong else np.arange(n_all)
    if strong and deal > 1:
        host = np.concatenate([full[int(all_offs[i]):int(all_offs[i + 1])] for i in mine]) if mine.size else full[:0]
    else:
        host = full
    my_size = int(host.size)
    lens_in = (all_offs[1:] - all_offs[:-1])[mine]
    n = int(mine.size)
    offs = np.zeros(n + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens_in)
    d_in = torch.from_numpy(np.ascontiguousarray(host)).to(D.dev)
    caps = np.array([lzma_amd.enc_bound(int(x)) for x in lens_in], dtype=np.uint64)
    cap_offs = np.zeros(n + 1, dtype=np.uint64)
    cap_offs[1:] = np.cumsum(caps)
    d_comp = torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=D.dev)
    d_comps = [d_comp]   # the unfenced split schedule codes batch j into d_comps[j % 2]
    d_packs = [torch.empty(int(cap_offs[-1]) + 1, dtype=torch.uint8, device=D.dev) for _ in range(2)]
    d_dec = torch.empty(my_size + 1, dtype=torch.uint8, device=D.dev)
    out_sizes = lens_in.astype(np.int64)
    props = lzma_amd.write_props(p)
    D.sync()   # the input copy above ran on the current stream
    state = {"dec_ok": True}
    # The parse of step k+1 waits for step k's decode when the streams fill the CUs (the
    # parser wants every stream resident from its start: 16 per CU at 4096). At <= 8 streams
    # per CU (strong-scaling shares) the parse and decode waves fit beside each other, so the
    # parse starts at once and step k's decode runs beside it.
    fence = overlap and n > 8 * D.cus()
    if fence:
        ctx.set_parse_fence(ctx_dec)
    lagged = overlap and args.pipeline == "split" and not fence
    if lagged:
        d_comps.append(torch.empty_like(d_comp))

    def check_dec(dlens, dstat):
        state["dec_ok"] &= bool((dstat == 0).all()) and bool((dlens == out_sizes).all())

    def decode(buf, pk):
        t1 = time.perf_counter()
        if overlap:
            ctx_dec.decode_batch_dev_async(props, buf, pk, out_sizes, d_dec, offs, st_dec)
            state["dec_inflight"] = True
        else:
            check_dec(*ctx_dec.decode_batch_dev(props, buf, pk, out_sizes, d_dec, offs, st_dec))
        state["t_dec"] = state.get("t_dec", 0.0) + (time.perf_counter() - t1)

    def join():   # the previous step's decode (pipelined: with the fence, done by now)
        if state.pop("dec_inflight", False):
            check_dec(*ctx_dec.decode_batch_dev_wait())

    def stage():
        ctx.encode_stage_dev(d_in, offs, p, d_comp, cap_offs, st)
        state["staged"] = state.get("staged", 0) + 1

    def step(k, ahead):   # ahead: the steps after this one in the same loop
        t0 = time.perf_counter()
        buf = d_packs[k % 2]
        if overlap and args.pipeline == "split" and fence:
            # 16 streams per CU: the parser fills the CUs and waits for step k-1's decode.
            # Step k's walk and parser on st, its range coder on the encoder context's coder
            # stream; step k+1's keys and sorts are staged behind the parser and run beside
            # that coder and step k's pack + decode (decoder context, st_dec)
            if not state.get("staged"):
                stage()
            ctx.encode_parse_dev_async(st)
            state["staged"] -= 1
            if ahead:
                stage()
            lens = ctx.encode_parse_dev_wait()
        if overlap and args.pipeline == "split":
            join()   # step k-1's decode (fenced: done, step k's parser waited for it)
            pk = ctx_dec.pack_dev(d_comp, cap_offs, lens, buf, st_dec)   # synchronous: buf is complete
        else:
            lens = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
            join()
            pk = ctx.pack_dev(d_comp, cap_offs, lens, buf, st)   # synchronous: buf is complete
        if dist:   # the single data exchange: rank 0 collects every rank's packed streams
            g, all_lens, counts = lzdist.gather_streams(buf, lens, dst=0)
            state["gathered"] = None if g is None else (g, all_lens, counts)
        state["lens"], state["pk"], state["buf"] = lens, pk, buf
        state["t_enc"] = state.get("t_enc", 0.0) + (time.perf_counter() - t0)
        join()
        decode(buf, pk)

    def finish(k, lens, t0):   # a lagged step's tail: pack + gather + decode of batch k
        buf = d_packs[k % 2]
        join()   # batch k-1's decode
        pk = ctx_dec.pack_dev(d_comps[k % 2], cap_offs, lens, buf, st_dec)   # synchronous: buf is complete
        if dist:
            g, all_lens, counts = lzdist.gather_streams(buf, lens, dst=0)
            state["gathered"] = None if g is None else (g, all_lens, counts)
        state["lens"], state["pk"], state["buf"] = lens, pk, buf
        state["t_enc"] = state.get("t_enc", 0.0) + (time.perf_counter() - t0)
        decode(buf, pk)

    def loop_lagged(nsteps):
        # <= 8 streams per CU, no parse fence: two batches staged and two range coders in
        # flight (one per live slot). On st: parser k, then batch k+2's keys and sorts, then
        # parser k+1 at once (enqueued before the host collects coder k, which runs beside
        # them); batch k+1's walk runs on the encoder context's walk stream beside parser k,
        # step k's pack + decode beside parser k+1. Batch j codes into d_comps[j % 2].
        def stage_j(j):
            ctx.encode_stage_dev(d_in, offs, p, d_comps[j % 2], cap_offs, st)
        if nsteps == 0:
            return
        stage_j(0)
        if nsteps > 1:
            stage_j(1)
        ctx.encode_parse_dev_async(st)
        if nsteps > 2:
            stage_j(2)
        for k in range(nsteps):
            t0 = time.perf_counter()
            if k + 1 < nsteps:
                ctx.encode_parse_dev_async(st)
                if k + 3 < nsteps:
                    stage_j(k + 3)
            finish(k, ctx.encode_parse_dev_wait(), t0)

    def barrier():
        if dist:
            torch.distributed.barrier()
        D.sync()

    # every step stages the next one inside its own time; the last step of each loop
    # stages nothing, so the timed loop holds exactly its own steps' work
    if lagged:
        loop_lagged(args.warmup)
    else:
        for k in range(args.warmup):
            step(k, args.warmup - 1 - k)
    join()
    for c in (ctx, ctx_dec):
        c.set_timing(True)
        c.reset_timings()
    state["t_enc"] = state["t_dec"] = 0.0
    barrier()
    t0 = time.perf_counter()
    if lagged:
        loop_lagged(args.steps)
    else:
        for k in range(args.steps):
            step(k, args.steps - 1 - k)
    join()
    barrier()
    elapsed = time.perf_counter() - t0
    if fence:
        ctx.set_parse_fence(None)
    if overlap:
        # the phases overlap: their MB/s come from the summed kernel times (HIP events)
        state["t_dec"] = sum(v[0] for k_, v in ctx_dec.timings().items()) / 1e3
        state["t_enc"] = sum(v[0] for k_, v in ctx.timings().items()) / 1e3
    timings = ctx.timings()
    timings.update(ctx_dec.timings())
    for c in (ctx, ctx_dec):
        c.set_timing(False)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=D.dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    comp_bytes = int(np.sum(state["lens"]))
    roundtrip = state["dec_ok"]
    if not args.no_verify:
        roundtrip = roundtrip and bool(torch.equal(d_dec[:my_size], d_in))
    gathered = None
    if dist:
        # the gather's check (after the timed loop): every rank's per-stream CRC-32 of what it
        # packed, against the streams rank 0 received; then the multi-member container
        import zlib
        host_pack = state["buf"][:comp_bytes].cpu().numpy()
        pk = state["pk"]
        mine_crc = [zlib.crc32(host_pack[int(pk[i]):int(pk[i + 1])]) for i in range(n)]
        every = [None] * world
        torch.distributed.all_gather_object(every, mine_crc)
        if rank == 0:
            g, all_lens, counts = state["gathered"]
            gb = g.cpu().numpy()
            goffs = np.concatenate([[0], np.cumsum(all_lens)]).astype(np.int64)
            got_crc = [zlib.crc32(gb[int(goffs[k]):int(goffs[k + 1])]) for k in range(len(all_lens))]
            want_crc = [c for per in every for c in per]
            order = lzdist.stream_order(counts, world) if strong else np.arange(len(all_lens))
            members = lzdist.reorder_payloads(gb.tobytes(), all_lens, order)
            sizes = ([int(all_offs[i + 1] - all_offs[i]) for i in range(n_all)] if strong
                     else [int(x) for x in np.tile(all_offs[1:] - all_offs[:-1], world)])
            blob = lzdist.pack_container(props, members, sizes)
            expect = n_all if strong else n_all * world
            back = lzdist.unpack_container(blob)
            gathered = {"bytes": int(g.numel()), "streams": len(back), "streams_expected": expect,
                        "crc_match": got_crc == want_crc,
                        "complete": len(back) == expect and got_crc == want_crc}
            if strong and args.dump_container:
                with open(args.dump_container, "wb") as f:
                    f.write(blob)
    # one buffer encoded, packed and decoded back to back (no pipelining): what a single
    # step costs on its own, reported beside the pipelined steady-state value
    # Its kernels are timed with HIP events and the library's host-side stalls (buffer
    # reallocations, whole-device syncs) counted, so the line shows where its time goes
    for c in (ctx, ctx_dec):
        c.set_timing(True)
        c.reset_timings()
    stats0 = [c.stats() for c in (ctx, ctx_dec)]
    barrier()
    t1 = time.perf_counter()
    lens1 = ctx.encode_batch_dev(d_in, offs, p, d_comp, cap_offs, st)
    t_e = time.perf_counter()
    pk1 = ctx.pack_dev(d_comp, cap_offs, lens1, d_packs[0], st)
    t_p = time.perf_counter()
    dl1, ds1 = ctx_dec.decode_batch_dev(props, d_packs[0], pk1, out_sizes, d_dec, offs, st_dec)
    barrier()
    seq_elapsed = time.perf_counter() - t1
    seq_wall = {"encode_ms": (t_e - t1) * 1e3, "pack_ms": (t_p - t_e) * 1e3, "decode_ms": (t1 + seq_elapsed - t_p) * 1e3}
    seq_kernels = ctx.timings()
    seq_kernels.update(ctx_dec.timings())
    seq_stats = {}
    for name, c, s0 in (("encoder", ctx, stats0[0]), ("decoder", ctx_dec, stats0[1])):
        s1 = c.stats()
        seq_stats[name] = {k: s1[k] - s0[k] for k in s1}
    for c in (ctx, ctx_dec):
        c.set_timing(False)
    seq_ok = bool((ds1 == 0).all()) and bool((dl1 == out_sizes).all()) and bool(np.array_equal(lens1, state["lens"]))
    if dist:
        t = torch.tensor([seq_elapsed], dtype=torch.float64, device=D.dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        seq_elapsed = float(t.item())
    return {"elapsed": elapsed, "timings": timings, "state": state, "host": host, "full": full, "offs": offs,
            "seq_elapsed": seq_elapsed, "seq_ok": seq_ok, "fence": fence, "seq_wall": seq_wall,
            "seq_kernels": seq_kernels, "seq_stats": seq_stats,
            "n": n, "n_all": n_all, "size": size, "my_size": my_size, "comp_bytes": comp_bytes,
            "roundtrip": roundtrip, "t_enc": state["t_enc"], "t_dec": state["t_dec"], "gathered": gathered,
            "bufs": (d_in, d_comp, d_packs, d_dec)}


def verify_parity(args, r, p, rank, world, dist, D, sample_idx=None):
    """Oracle parity of the pass's streams (after the timed region). Returns (cpu_baseline
    block or None, ok, streams checked)."""
    cpu, ref = None, {}
    n, offs, host = r["n"], r["offs"], r["host"]
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import oracle_ffi as orc
    op = orc.params(p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos)
    chunks = [host[int(offs[i]):int(offs[i + 1])] for i in range(n)]
    if rank == 0 and world == 1 and args.cpu_sample > 0 and sample_idx is None:
        cpu, ref = cpu_baseline(orc, op, chunks, args)
    if not args.no_verify:
        if sample_idx is not None:
            want = sample_idx
        else:
            want = range(n) if args.parity_streams < 0 else spread(n, args.parity_streams)
        idx = [i for i in want if i not in ref]
        if idx:   # not timed: the parity check of the streams the baseline sample did not cover
            outs = orc.encode_many([chunks[i].tobytes() for i in idx], op, threads=orc.cpu_threads())
            ref.update(zip(idx, outs))
    ok, checked = True, 0
    if ref:
        host_pack = r["state"]["buf"][:r["comp_bytes"]].cpu().numpy()
        pk = r["state"]["pk"]
        for i, b in ref.items():
            checked += 1
            if host_pack[int(pk[i]):int(pk[i + 1])].tobytes() != b:
                ok = False
    ok = ok and r["roundtrip"] and (checked > 0 or args.no_verify)
    if r["gathered"] is not None:
        ok = ok and r["gathered"]["complete"]
    if dist:
        flag = torch.tensor([1 if ok else 0, checked], device=D.dev, dtype=torch.int64)
        torch.distributed.all_reduce(flag[:1], op=torch.distributed.ReduceOp.MIN)
        torch.distributed.all_reduce(flag[1:], op=torch.distributed.ReduceOp.SUM)
        ok, checked = bool(flag[0].item()), int(flag[1].item())
    return cpu, ok, checked, (orc, op)


def main():
    args = parse()
    if args.emulate:
        os.environ.setdefault("LZMA_AMD_LIB", SIMT_LIB)
        lzma_amd.LIB_PATH = os.environ["LZMA_AMD_LIB"]
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    D = Device(args.emulate, local)
    if dist:
        import torch.distributed as td
        if args.emulate:
            td.init_process_group("gloo")
        else:
            td.init_process_group("nccl", device_id=D.dev)
        world = td.get_world_size()   # n_gpus comes from the process group
        rank = td.get_rank()
    dict_log = args.dict_log if args.dict_log is not None else (28 if args.data == "text" else 26)
    p = lzma_amd.make_params(dict_size=1 << dict_log, fb=32, mf=1, lc=3, lp=0, pb=2)
    ctx = lzma_amd.Context(D.index)
    ctx.set_batch_bytes(args.batch_bytes)
    ctx_dec = lzma_amd.Context(D.index)   # the decoder: its own context (device workspace) and HIP stream
    ctxs = (ctx, ctx_dec, D.new_stream(), D.new_stream())

    # ---- strong scaling: one --size buffer, streams dealt round-robin (value)
    r = run_pass(args, D, p, ctxs, True, rank, world, dist)
    cpu, ok, checked, (orc, op) = verify_parity(args, r, p, rank, world, dist, D)
    weak = None
    if dist and not args.no_weak:
        del r["bufs"]
        w = run_pass(args, D, p, ctxs, False, rank, world, dist)
        wn = w["n"]
        _, wok, wchecked, _ = verify_parity(args, w, p, rank, world, dist, D, sample_idx=spread(wn, 32))
        weak = {"value": w["size"] * world * args.steps / w["elapsed"] / 1e6, "unit": "MB/s",
                "ms_per_step": w["elapsed"] / args.steps * 1e3, "bytes_per_gpu": w["my_size"],
                "streams_per_gpu": wn, "verified": wok, "parity_streams_checked": wchecked,
                "gathered": w["gathered"],
                "kernels_ms": {k: {"total_ms": v[0], "launches": v[1]} for k, v in w["timings"].items()}}
        del w

    single = None
    if rank == 0 and world == 1 and args.single_stream > 0 and not args.emulate:
        single = single_stream(args, r["full"], p, D.dev, ctxs[2], orc, op)

    elapsed, timings, size, my_size, n, n_all = r["elapsed"], r["timings"], r["size"], r["my_size"], r["n"], r["n_all"]
    comp_bytes = r["comp_bytes"]
    value = size * args.steps / elapsed / 1e6   # the one buffer's bytes per max-over-ranks step time

    # ---- roofline for the dominant kernel (HIP events on the launch stream)
    dom = max(timings.items(), key=lambda kv: kv[1][0]) if timings else ("none", (0.0, 1))
    dname, (dms, dlaunch) = dom
    avg_s = dms / 1e3 / max(dlaunch, 1)
    per_step_launches = max(dlaunch // max(args.steps, 1), 1)
    # compress: N_in + N_out per launch; decompress: N_comp + N_out (the same two numbers)
    alg = (my_size + comp_bytes) / per_step_launches
    achieved = alg / avg_s if avg_s > 0 else 0.0
    wl = {"bytes_per_gpu": args.size, "chunk": args.chunk, "data": args.data, "dict_log": dict_log}
    traffic, traffic_src = pmc_traffic(dname, wl)
    roofline = {"bound": "hbm", "kernel": dname, "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                "unit": "GB/s", "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_source": traffic_src,
                "avg_launch_ms": avg_s * 1e3, "launches_per_step": per_step_launches,
                "alg_bytes_per_launch": alg, "issue": issue_bound(dname, wl, avg_s, my_size)}

    t_enc, t_dec = r["t_enc"], r["t_dec"]
    ratio = comp_bytes / max(my_size, 1)
    if rank == 0:
        desc = "LzmaBench generator" if args.data == "bench" else "TEXT (enwik9-shaped) generator"
        chunking = {"chunk_KiB": args.chunk >> 10, "ratio_chunked": ratio,
                    "note": "configs 2/3 run as independent %d KiB streams (SURVEY 8(d) stream rule); the output "
                            "is that many bytes larger than one whole-buffer stream would be" % (args.chunk >> 10)}
        if single is not None:
            chunking["ratio_one_stream"] = single["ratio"]
            chunking["one_stream_bytes"] = single["bytes"]
            chunking["extra_output_frac"] = ratio / single["ratio"] - 1 if single["ratio"] else None
        res = {
            "metric": "compress+decompress MB/s on 1 GB synthetic; bit-exact .lzma vs Java ref",
            "value": value, "unit": "MB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (%s)%s" % (desc, "; CPU SIMT emulation, not a measurement" if args.emulate else ""),
            "config": {"workload": "%s %d MiB as %d independent streams of %g KiB dealt round-robin over the GPUs; "
                                   "dict 2^%d fb32 bt4 lc3 lp0 pb2 (level-5 mapping); encode+pack+decode"
                                   % (desc, size >> 20, n_all, args.chunk / 1024, dict_log),
                       "bytes_per_gpu": my_size, "chunk": args.chunk, "streams_per_gpu": n,
                       "parallelism": "independent streams, %d rank(s), round-robin" % world},
            "compress_MBps": size * args.steps / max(t_enc, 1e-9) / 1e6,
            "decompress_MBps": size * args.steps / max(t_dec, 1e-9) / 1e6,
            "schedule": ("sequential: each step's encode and decode back to back; compress/decompress MB/s are "
                         "each phase's wall time (rank 0)") if args.sequential else
                        ("pipelined (%s): step k's %sdecode (own context + HIP stream) runs beside step k+1's "
                         "match finder, step k+1's parser waits for the decode; compress/decompress MB/s are each "
                         "phase's summed kernel times (HIP events), which overlap" % (
                             args.pipeline, "range coder (the encoder's coder stream), pack and "
                             if args.pipeline == "split" else "")),
            "sequential": {"value": size / r["seq_elapsed"] / 1e6, "unit": "MB/s", "ms": r["seq_elapsed"] * 1e3,
                           "lengths_equal_timed_steps": r["seq_ok"], "wall_ms": r["seq_wall"],
                           "kernels_ms": {k: {"total_ms": v[0], "launches": v[1]} for k, v in r["seq_kernels"].items()},
                           "library_stalls": r["seq_stats"],
                           "note": "one buffer encoded, packed and decoded back to back after the timed loop (no "
                                   "pipelining): the cost of one step on its own; value is the pipelined steady state. "
                                   "kernels_ms: HIP events on the launch streams; library_stalls: the library's "
                                   "buffer reallocations and whole-device syncs during the leg (lzma_ctx_stats)"},
            "parse_fence": r["fence"],
            "ratio": ratio, "chunking": chunking, "verified": ok,
            "verified_means": "every stream decodes to its input and every sampled stream's bytes equal the "
                              "oracle's Encoder.Code restatement%s" % (
                                  "; rank 0's gathered container holds every stream" if dist else ""),
            "parity_streams_checked": checked, "roundtrip_ok": r["roundtrip"],
            "projection_of_n_gpus": args.project_share if args.project_share > 1 else None,
            "gathered": r["gathered"], "weak_scaling": weak,
            "kernels_ms": {k: {"total_ms": v[0], "launches": v[1]} for k, v in timings.items()},
            "roofline": roofline, "cpu_baseline": cpu, "single_stream": single,
        }
        print(json.dumps(res), flush=True)
    if weak is not None:
        ok = ok and weak["verified"]
    ctx.close()
    ctx_dec.close()
    if dist:
        torch.distributed.destroy_process_group()
    if not ok:
        sys.exit(1)


# HIP-event timing label -> rocprofv3 kernel-name prefix
_KERNEL_OF = {"enc_parse": "enc_kernel", "dec_stream": "dec_kernel", "mf_walk": "mf_walk_kernel"}


def _profile_prefix(wl):
    """round 6's summaries (tools/r06/prof.sh, DATA=bench / DATA=text) of this same
    workload, taken at the kernels this tree builds"""
    return "r06/text_" if wl.get("data") == "text" else "r06/"


def _profile(name, wl):
    """A committed per-kernel summary from profiles/ (written by tools/r06/prof.sh
    over this same workload), or None when absent or taken on another workload."""
    path = os.path.join(REPO, "profiles", _profile_prefix(wl) + name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        t = json.load(f)
    meta = t.get("_workload", {})
    for k, v in wl.items():
        if meta.get(k, {"data": "bench", "dict_log": 26}.get(k)) != v:
            return None
    return t


def pmc_traffic(label, wl):
    """HBM bytes per launch of the dominant kernel from profiles/traffic.json
    (separate FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled per the gfx950
    correction of MI355X_MICROARCH.md)."""
    t = _profile("traffic.json", wl)
    if t is None:
        return None, None
    prefix = _KERNEL_OF.get(label, label)
    for k, v in t.items():
        if k.startswith(prefix) and isinstance(v, dict) and "traffic_bytes_per_launch" in v:
            return v["traffic_bytes_per_launch"], "profiles/%straffic.json (%s, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE)" % (
                _profile_prefix(wl), k)
    return None, None


def issue_bound(label, wl, avg_s, nbytes):
    """The scalar-issue bound of the dominant kernel (the CU's single
    scalar unit, not HBM, bounds the per-stream kernels): SQ_INSTS_SALU per CU over
    (clock x kernel time), and instructions per input byte, from profiles/issue.json
    (rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU ... over this workload)."""
    t = _profile("issue.json", wl)
    if t is None:
        return None
    prefix = _KERNEL_OF.get(label, label)
    for k, v in t.items():
        if k.startswith(prefix) and isinstance(v, dict) and "SQ_INSTS_SALU" in v:
            cus, clk = t.get("_cus", 256), t.get("_sclk_hz", 2.4e9)
            salu = v["SQ_INSTS_SALU"]
            insts = v.get("SQ_INSTS_SALU", 0) + v.get("SQ_INSTS_VALU", 0) + v.get("SQ_INSTS_LDS", 0) + \
                v.get("SQ_INSTS_VMEM", 0) + v.get("SQ_INSTS_SMEM", 0) + v.get("SQ_INSTS_BRANCH", 0)
            return {"salu_per_cu": salu / cus, "salu_issue_frac": salu / cus / (clk * avg_s) if avg_s > 0 else None,
                    "salu_per_input_byte": salu / max(nbytes, 1), "insts_per_input_byte": insts / max(nbytes, 1),
                    "clock_hz": clk, "source": "profiles/%sissue.json (%s)" % (_profile_prefix(wl), k)}
    return None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(orc, op, chunks, args):
    """The oracle (bit-exact C restatement of Encoder.Code / Decoder.Code; there is
    no JDK on the box) on a bounded sample of the same streams, as
    SURVEY 8(d) prescribes: (i) 1 thread, (ii) the job's CPU share, one reused
    encoder instance per thread (BinTree.Init clears the hash per Code call,
    BinTree.java:72-80). MB/s of uncompressed bytes, encode then decode. Returns
    the baseline block and the oracle bytes per sampled stream (the parity sample)."""
    from concurrent.futures import ThreadPoolExecutor
    props = orc.props(op)
    n = len(chunks)
    chunk = args.chunk

    def run(idx, threads):
        data = [chunks[i].tobytes() for i in idx]
        nbytes = sum(len(d) for d in data)
        t0 = time.perf_counter()
        encs = orc.encode_many(data, op, threads=threads)
        t1 = time.perf_counter()

        def dec(pair):
            c, e = pair
            rc, d = orc.decode(e, props, len(c))
            return rc == 1 and d == c
        with ThreadPoolExecutor(max_workers=threads) as ex:
            good = all(ex.map(dec, zip(data, encs)))
        t2 = time.perf_counter()
        if not good:
            raise RuntimeError("oracle round trip failed")
        return encs, {"value": nbytes / (t2 - t0) / 1e6, "compress_MBps": nbytes / (t1 - t0) / 1e6,
                      "decompress_MBps": nbytes / (t2 - t1) / 1e6, "bytes": nbytes, "streams": len(idx)}

    nproc = os.cpu_count() or 1
    quota = cgroup_cpus()
    named = {"share": quota or orc.cpu_threads(), "node_share": max(1, nproc // 8), "nproc": nproc}
    counts = []
    for t in args.cpu_threads.split(","):
        t = t.strip()
        c = named[t] if t in named else int(t)
        if c not in counts:
            counts.append(c)
    one_idx = spread(n, max(1, args.cpu_single // chunk))
    _, one = run(one_idx, 1)
    multi_idx = spread(n, max(1, args.cpu_sample // chunk))
    by_threads, encs = {}, None
    for c in counts:
        e, r = run(multi_idx, c)
        encs = encs or e
        by_threads[str(c)] = r
    best = max(by_threads, key=lambda k: by_threads[k]["value"])
    multi = by_threads[best]
    res = {"value": multi["value"], "unit": "MB/s", "cores": int(best), "kind": "port",
           "compress_MBps": multi["compress_MBps"], "decompress_MBps": multi["decompress_MBps"],
           "cpu_model": cpu_model(), "cpus_visible": nproc, "cgroup_cpu_quota": quota,
           "node_share_cpus": named["node_share"],
           "by_threads": {k: {"value": v["value"], "compress_MBps": v["compress_MBps"],
                              "decompress_MBps": v["decompress_MBps"]} for k, v in by_threads.items()},
           "single_thread": dict(one, cores=1),
           "sample": "%d of the %d streams (%d MiB, spread evenly over the buffer), oracle/ C restatement of the "
                     "Java reference (no JDK on the box), one reused encoder per thread, timed at %s threads "
                     "(the job's cgroup CPU quota, nproc / 8 and nproc); value = the fastest (%s threads); "
                     "single_thread: %d streams on 1 thread"
                     % (len(multi_idx), n, multi["bytes"] >> 20, "/".join(str(c) for c in counts), best,
                        len(one_idx))}
    return res, dict(zip(multi_idx, encs))


def cgroup_cpus():
    """CPUs the job may use per the cgroup quota (cpu.max 'quota period'), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return None


def single_stream(args, full, p, dev, st, orc, op):
    """SURVEY 7.3's serial tail (config 4's regime: one stream far longer than a chunk): one
    stream of --single-stream bytes of the same data, dict as the workload, encoded and decoded
    on the GPU (device-resident, one wave parses it), beside the oracle on one
    host thread on the same bytes; the GPU bytes must equal the oracle's."""
    n = min(args.single_stream, full.size)
    host = full[:n]
    d_in = torch.from_numpy(host).to(dev)
    cap = lzma_amd.enc_bound(n)
    d_out = torch.empty(cap + 1, dtype=torch.uint8, device=dev)
    d_dec = torch.empty(n + 1, dtype=torch.uint8, device=dev)
    ctx = lzma_amd.Context(dev.index)
    ctx.set_batch_bytes(max(n, 1 << 20))
    ctx.set_timing(True)
    offs = np.array([0, n], dtype=np.uint64)
    coffs = np.array([0, cap], dtype=np.uint64)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    lens = ctx.encode_batch_dev(d_in, offs, p, d_out, coffs, st)
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    dl, ds = ctx.decode_batch_dev(lzma_amd.write_props(p), d_out, np.array([0, int(lens[0])], dtype=np.uint64),
                                  np.array([n], dtype=np.int64), d_dec, offs, st)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    tm = ctx.timings()
    ctx.close()
    enc = d_out[:int(lens[0])].cpu().numpy().tobytes()
    ok = int(ds[0]) == 0 and int(dl[0]) == n and bool(torch.equal(d_dec[:n], d_in))
    res = {"bytes": int(n), "dict_log": int(p.dict_size).bit_length() - 1, "gpu_compress_MBps": n / (t1 - t0) / 1e6,
           "gpu_decompress_MBps": n / (t2 - t1) / 1e6, "parse_ms": tm.get("enc_parse", (0.0, 0))[0],
           "parse_cycles_per_byte": tm.get("enc_parse", (0.0, 0))[0] / 1e3 * 2.4e9 / max(n, 1),
           "ratio": len(enc) / max(n, 1), "roundtrip_ok": ok,
           "projected_1GiB_encode_s": (1 << 30) / max(n / (t1 - t0), 1e-9)}
    if orc is not None:
        data = host.tobytes()
        c0 = time.perf_counter()
        ref = orc.EncoderSession(op).encode(data)
        c1 = time.perf_counter()
        rc, back = orc.decode(ref, orc.props(op), n)
        c2 = time.perf_counter()
        res.update(cpu_1thread_compress_MBps=n / (c1 - c0) / 1e6, cpu_1thread_decompress_MBps=n / (c2 - c1) / 1e6,
                   equals_oracle=ref == enc, gpu_over_cpu_compress=(c1 - c0) / (t1 - t0))
    return res


if __name__ == "__main__":
    main()
