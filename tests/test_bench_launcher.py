"""bench.py's multi-GPU launcher on CPU: `bench.py --gpus 2`
without WORLD_SIZE starts two rank processes itself; with --emulate they use gloo
and the product kernels compiled for the CPU SIMT emulation (tests/simt). The
strong pass deals one buffer's streams round-robin ({i : i mod 2 = r}); rank 0
gathers every rank's packed streams, and the multi-member container it writes must
hold every stream, each equal to the oracle's Encoder.Code bytes."""
import json
import os
import subprocess
import sys

import pytest

import oracle_ffi as orc
from lzma_amd import dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMT = os.path.join(REPO, "tests", "simt")


@pytest.mark.timeout(900)
@pytest.mark.parametrize("steps,warmup", [(1, 0), (4, 2)])
def test_bench_gpus2_launcher_emulated(tmp_path, steps, warmup):
    """steps 4 / warmup 2: the lagged split schedule (no parse fence at these stream counts:
    two batches staged, two range coders in flight) over several steps, verified."""
    subprocess.check_call(["make", "-s", "-j", "8", "-C", SIMT, "so"])
    cont = str(tmp_path / "gathered.lzmg")
    size, chunk = 40000, 5000
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--emulate",
                          "--size", str(size), "--chunk", str(chunk), "--steps", str(steps), "--warmup", str(warmup),
                          "--cpu-sample", "0", "--single-stream", "0", "--dump-container", cont],
                         env=env, capture_output=True, text=True, timeout=800)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-3000:]   # ONE JSON line, from rank 0
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["scaling"] == "strong" and res["verified"]
    assert res["sequential"]["lengths_equal_timed_steps"] and res["parse_fence"] is False
    n_all = (size + chunk - 1) // chunk
    assert res["config"]["streams_per_gpu"] == n_all // 2
    g = res["gathered"]
    assert g["streams"] == g["streams_expected"] == n_all and g["crc_match"] and g["complete"]
    w = res["weak_scaling"]
    assert w["verified"] and w["gathered"]["streams"] == 2 * n_all
    # the gathered container: every stream of the buffer, in order, equal to the oracle's bytes
    import lzma_amd
    data = lzma_amd.bench_generate(size).tobytes()
    members = dist.unpack_container(open(cont, "rb").read())
    assert len(members) == n_all
    op = orc.params(1 << 26, 32, 1, 3, 0, 2, 0)
    for i, m in enumerate(members):
        s = data[i * chunk:(i + 1) * chunk]
        assert m[:5] == orc.props(op) and int.from_bytes(m[5:13], "little") == len(s)
        assert m[13:] == orc.encode(s, op)
