"""Config 4's stream on one MI355X: ONE 1 GiB BENCH stream (LzmaBench generator, dict 2^26,
fb 32, BT4, lc3 lp0 pb2) encoded as Encoder.Code would (Encoder.java:1064-1077), through the
sliced encode (lzma_enc_session_*) across several processes: the serial parse of that stream
is ~30 minutes and one gpurun call is at most 20. Each call recomputes the match finder (a
pure function of the input), restores the checkpoint the last call left, steps slices until
its time budget and checkpoints again. The output bytes are hashed (SHA-256) in 4 MiB blocks as
they become final; tools/r06/config4_check.py compares the blocks with the oracle's output.

usage (on the GPU box): python tools/r06/config4_sliced.py --state-in DIR --state-out DIR
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
import lzma_amd  # noqa: E402

BLOCK = 4 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mib", type=int, default=1024)
    ap.add_argument("--slice", type=int, default=16 << 20, help="input bytes per launch")
    ap.add_argument("--budget", type=float, default=1000.0, help="seconds of stepping in this call")
    ap.add_argument("--state-in", default=None)
    ap.add_argument("--state-out", required=True)
    a = ap.parse_args()
    t_start = time.time()
    n = a.mib << 20
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32, mf=1, lc=3, lp=0, pb=2)
    blob, log, tail = None, {"mib": a.mib, "block": BLOCK, "hashes": [], "calls": []}, b""
    if a.state_in and os.path.exists(os.path.join(a.state_in, "session.blob")):
        with open(os.path.join(a.state_in, "session.blob"), "rb") as f:
            blob = f.read()
        with open(os.path.join(a.state_in, "log.json")) as f:
            log = json.load(f)
        with open(os.path.join(a.state_in, "tail.bin"), "rb") as f:
            tail = f.read()
        assert log["mib"] == a.mib and log["block"] == BLOCK
    data = lzma_amd.bench_generate(n)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    d_in = torch.from_numpy(data).to(dev)
    cap = lzma_amd.enc_bound(n)
    d_out = torch.zeros(cap + 1, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize(dev)
    ctx = lzma_amd.Context(0)
    ctx.set_batch_bytes(max(1 << 30, n))
    t0 = time.time()
    s = ctx.session(d_in, n, p, d_out, cap, st, resume=blob)
    t_mf = time.time() - t0
    in0, out0 = s.in_pos, s.out_len
    print("call %d: match finder + restore %.1f s, resuming at input %d, output %d" % (
        len(log["calls"]), t_mf, in0, out0), flush=True)
    steps, t_step, last = 0, 0.0, 0.0
    while not s.done and (time.time() - t_start) + 1.5 * last < a.budget:
        prev_in, prev_out = s.in_pos, s.out_len
        t1 = time.time()
        s.step(a.slice)
        last = time.time() - t1
        t_step += last
        steps += 1
        tail += d_out[prev_out:s.out_len].cpu().numpy().tobytes()
        while len(tail) >= BLOCK:
            log["hashes"].append(hashlib.sha256(tail[:BLOCK]).hexdigest())
            tail = tail[BLOCK:]
        print("slice %d: input %d -> %d (%.3f MB/s), output %d, %.1f s elapsed" % (
            steps, prev_in, s.in_pos, (s.in_pos - prev_in) / max(last, 1e-9) / 1e6, s.out_len,
            time.time() - t_start), flush=True)
    if s.done and tail:
        log["hashes"].append(hashlib.sha256(tail).hexdigest())
        log["last_block_bytes"] = len(tail)
        tail = b""
    log["calls"].append({"match_finder_restore_s": t_mf, "slices": steps, "step_s": t_step, "in_from": in0,
                         "in_to": s.in_pos, "out_to": s.out_len,
                         "parse_MBps": (s.in_pos - in0) / max(t_step, 1e-9) / 1e6, "done": s.done})
    log.update(in_pos=s.in_pos, out_len=s.out_len, done=s.done, n=n)
    os.makedirs(a.state_out, exist_ok=True)
    if not s.done:
        with open(os.path.join(a.state_out, "session.blob"), "wb") as f:
            f.write(s.save())
    with open(os.path.join(a.state_out, "tail.bin"), "wb") as f:
        f.write(tail)
    with open(os.path.join(a.state_out, "log.json"), "w") as f:
        json.dump(log, f, indent=1)
    s.close()
    ctx.close()
    print(json.dumps(log["calls"][-1]), flush=True)


if __name__ == "__main__":
    main()
