"""The oracle side of config 4's sliced run (tools/r06/config4_sliced.py): the oracle's
Encoder.Code restatement over the same 1 GiB BENCH stream, its output hashed in the same 4 MiB
blocks (written once to profiles/r06/config4_oracle_blocks.json, about 5 minutes on one host
core), then compared block by block with a GPU run's log.json.

usage: python tools/r06/config4_check.py [GPU_LOG_JSON]"""
import hashlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "lzma-java_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import lzma_amd  # noqa: E402
import oracle_ffi as orc  # noqa: E402

REF = os.path.join(REPO, "profiles", "r06", "config4_oracle_blocks.json")
BLOCK = 4 << 20


def oracle_blocks(mib=1024):
    if os.path.exists(REF):
        with open(REF) as f:
            return json.load(f)
    n = mib << 20
    data = lzma_amd.bench_generate(n).tobytes()
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32, mf=1, lc=3, lp=0, pb=2)
    t0 = time.time()
    out = orc.EncoderSession(orc.params(p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos)).encode(data)
    t = time.time() - t0
    r = {"mib": mib, "block": BLOCK, "out_len": len(out), "md5": hashlib.md5(out).hexdigest(),
         "oracle_s": t, "hashes": [hashlib.sha256(out[i:i + BLOCK]).hexdigest() for i in range(0, len(out), BLOCK)]}
    with open(REF, "w") as f:
        json.dump(r, f, indent=1)
    return r


def main():
    ref = oracle_blocks()
    print("oracle: %d bytes, %d blocks, md5 %s" % (ref["out_len"], len(ref["hashes"]), ref["md5"]))
    if len(sys.argv) > 1:
        with open(sys.argv[1]) as f:
            g = json.load(f)
        k = len(g["hashes"])
        same = g["hashes"] == ref["hashes"][:k]
        print("gpu: %d blocks final (output %d bytes, input %d of %d, done %s): %s" % (
            k, g["out_len"], g["in_pos"], g["n"], g["done"], "EQUAL to the oracle's first %d blocks" % k if same
            else "DIFFERENT at block %d" % next(i for i in range(k) if g["hashes"][i] != ref["hashes"][i])))
        if g["done"]:
            print("complete stream: %s" % ("byte-equal (every block, length %d)" % g["out_len"]
                                          if same and k == len(ref["hashes"]) and g["out_len"] == ref["out_len"]
                                          else "MISMATCH"))


if __name__ == "__main__":
    main()
