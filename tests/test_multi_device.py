"""The multi-device batch entry points (lzma_mctx, SURVEY 8(b) device_mask).

CPU: the product sources compiled for the SIMT emulation with two emulated
devices (HIPEMU_DEVICES=2), in a subprocess: streams dealt round-robin over
the two devices, each on its own host thread and context, must come back in
stream order and equal the oracle's bytes. GPU: every visible device."""
import os
import subprocess
import sys

import numpy as np
import pytest

import lzma_amd
import oracle_ffi as orc

HERE = os.path.dirname(os.path.abspath(__file__))
SIMT = os.path.join(HERE, "simt")

_CHILD = r"""
import sys
sys.path.insert(0, %(pkg)r); sys.path.insert(0, %(tests)r)
import numpy as np, lzma_amd, oracle_ffi as orc
lzma_amd.LIB_PATH = %(lib)r
data = lzma_amd.text_generate(7 * 5000 + 321).tobytes()
streams = [data[i:i + 5000] for i in range(0, len(data), 5000)] + [b"", b"x"]
p = lzma_amd.make_params(dict_size=1 << 20, fb=48)
m = lzma_amd.MultiContext(0b11)
assert m.devices == 2
outs = m.encode_batch(streams, p)
op = orc.params(1 << 20, 48, 1, 3, 0, 2, 0)
for i, (s, o) in enumerate(zip(streams, outs)):
    assert o == orc.encode(s, op), i
dec = m.decode_batch(outs, lzma_amd.write_props(p), [len(s) for s in streams])
for s, (st, d) in zip(streams, dec):
    assert st == 0 and d == s
m.close()
try:
    lzma_amd.MultiContext(0b100)   # device 2 is not there
    raise SystemExit("expected an error")
except lzma_amd.LzmaError:
    pass
print("multi ok")
"""


@pytest.mark.timeout(300)
def test_multi_device_round_robin_emulated_two_devices():
    subprocess.check_call(["make", "-s", "-j", "8", "-C", SIMT, "so"])
    code = _CHILD % {"pkg": os.path.join(os.path.dirname(HERE), "lzma-java_amd"), "tests": HERE,
                     "lib": os.path.join(SIMT, "build", "so", "libsimt_lzma.so")}
    env = dict(os.environ, HIPEMU_DEVICES="2")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=280)
    assert r.returncode == 0 and "multi ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.gpu
def test_multi_device_all_visible_gpus():
    torch = pytest.importorskip("torch")
    ndev = torch.cuda.device_count()
    data = lzma_amd.bench_generate(3 << 20).tobytes()
    streams = [data[i:i + (200 << 10)] for i in range(0, len(data), 200 << 10)]
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32)
    m = lzma_amd.MultiContext((1 << ndev) - 1)
    try:
        outs = m.encode_batch(streams, p)
        ref = orc.encode_many(streams, orc.params(1 << 26, 32, 1, 3, 0, 2, 0))
        assert outs == ref
        dec = m.decode_batch(outs, lzma_amd.write_props(p), [len(s) for s in streams])
        assert all(st == 0 and d == s for s, (st, d) in zip(streams, dec))
    finally:
        m.close()
    with pytest.raises(lzma_amd.LzmaError):   # a device that is not there
        lzma_amd.MultiContext(1 << ndev)
