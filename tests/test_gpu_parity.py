"""GPU parity: the HIP path (through the C ABI) against the reference's golden
vectors and against the CPU restatement (oracle/) on seeded inputs.

Bar: bit-exact. Every encoded stream must equal Encoder.Code's bytes on the
same input and parameters; every decode must equal Decoder.Code's output and
status.
"""
import hashlib
import io
import json
import os

import numpy as np
import pytest

import lzma_amd
import oracle_ffi as orc

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def ctx():
    c = lzma_amd.Context(0)
    yield c
    c.close()


def _oparams(p):
    return orc.params(p.dict_size, p.fb, p.mf, p.lc, p.lp, p.pb, p.eos)


def _switch_params(switches):
    kw = dict(dict_size=1 << 23, fb=128, mf=1, lc=3, lp=0, pb=2, eos=0)   # LzmaAlone.java:24-37
    for s in switches:
        s = s[1:]
        if s.startswith("fb"):
            kw["fb"] = int(s[2:])
        elif s.startswith("lc"):
            kw["lc"] = int(s[2:])
        elif s.startswith("lp"):
            kw["lp"] = int(s[2:])
        elif s.startswith("pb"):
            kw["pb"] = int(s[2:])
        elif s == "eos":
            kw["eos"] = 1
        elif s == "mfbt2":
            kw["mf"] = 0
        elif s.startswith("d"):
            kw["dict_size"] = 1 << int(s[1:])
    return lzma_amd.make_params(**kw)


with open(os.path.join(GOLD, "lzma_alone_goldens.json")) as f:
    _GOLDENS = json.load(f)["cases"]


@pytest.fixture(scope="module")
def firefox():
    with open(os.path.join(GOLD, "firefox.exe"), "rb") as f:
        return f.read()


@pytest.mark.parametrize("case", _GOLDENS, ids=[" ".join(c["switches"]) or "default" for c in _GOLDENS])
def test_gpu_lzma_alone_golden(ctx, firefox, case):
    """LzmaAloneTest.java:25-39 on the GPU: md5 + length of the .lzma file and the round trip."""
    p = _switch_params(case["switches"])
    blob = lzma_amd.compress_file_bytes(firefox, p, ctx)
    assert len(blob) == case["len"]
    assert hashlib.md5(blob).hexdigest() == case["md5"]
    assert lzma_amd.decompress_file_bytes(blob, ctx) == firefox


def _inputs(rng):
    yield b""
    yield b"A"
    yield b"AB"
    yield b"ABC"
    yield b"\x00" * 7000
    yield rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    words = [b"alpha", b"beta", b"gamma", b"delta", b"the", b" ", b"\n", b"theta"]
    yield b"".join(words[i] for i in rng.integers(0, len(words), 5000))
    yield (b"abcdefghij" * 900)[:8999]
    yield rng.integers(0, 3, 30000, dtype=np.uint8).tobytes()
    yield lzma_amd.bench_generate(60000).tobytes()


_PARAMS = [
    dict(dict_size=1 << 26, fb=32, mf=1),                      # L5 mapping
    dict(dict_size=1 << 12, fb=5, mf=0),
    dict(dict_size=1 << 20, fb=273, mf=1, lc=0, lp=2, pb=0),
    dict(dict_size=100, fb=64, mf=2, eos=1),
    dict(dict_size=1, fb=16, mf=1),
    dict(dict_size=1 << 16, fb=48, mf=1, lc=8, lp=0, pb=4),   # literal coders in HBM (lc+lp > 3)
]


@pytest.mark.parametrize("pi", range(len(_PARAMS)))
def test_gpu_encode_matches_oracle(ctx, pi):
    p = lzma_amd.make_params(**_PARAMS[pi])
    rng = np.random.default_rng(100 + pi)
    streams = list(_inputs(rng))
    outs = ctx.encode_batch(streams, p)
    for i, (s, o) in enumerate(zip(streams, outs)):
        assert o == orc.encode(s, _oparams(p)), "stream %d (len %d)" % (i, len(s))


@pytest.mark.parametrize("pi", range(len(_PARAMS)))
def test_gpu_decode_matches_oracle(ctx, pi):
    p = lzma_amd.make_params(**_PARAMS[pi])
    rng = np.random.default_rng(200 + pi)
    streams = list(_inputs(rng))
    enc = [orc.encode(s, _oparams(p)) for s in streams]
    sizes = [-1 if p.eos else len(s) for s in streams]
    res = ctx.decode_batch(enc, lzma_amd.write_props(p), sizes, caps=[len(s) + 64 for s in streams])
    for s, (st, dec) in zip(streams, res):
        assert st == lzma_amd.LZMA_OK and dec == s


def test_gpu_many_streams_bench_chunks(ctx):
    """Config-5 shape in miniature: many independent BENCH chunks of ragged sizes, L5 params."""
    data = lzma_amd.bench_generate(3 << 20).tobytes()
    rng = np.random.default_rng(5)
    cuts = np.sort(rng.integers(0, len(data), 300))
    cuts = np.concatenate([[0], cuts, [len(data)]])
    streams = [data[cuts[i]:cuts[i + 1]] for i in range(len(cuts) - 1)]
    p = lzma_amd.make_params(dict_size=1 << 18, fb=32)
    outs = ctx.encode_batch(streams, p)
    for i in range(0, len(streams), 7):   # oracle on a deterministic subset keeps this test in seconds
        assert outs[i] == orc.encode(streams[i], _oparams(p)), i
    dec = ctx.decode_batch(outs, lzma_amd.write_props(p), [len(s) for s in streams])
    for s, (st, d) in zip(streams, dec):
        assert st == lzma_amd.LZMA_OK and d == s


def test_gpu_wide_pairs_stream_over_8mib(ctx):
    """A stream > 8 MiB switches match pairs to 64-bit packing."""
    data = lzma_amd.bench_generate(9 << 20).tobytes()
    p = lzma_amd.make_params(dict_size=1 << 24, fb=32)
    out = ctx.encode_batch([data], p)[0]
    assert out == orc.encode(data, _oparams(p))


def test_gpu_corrupt_streams_status_matches_oracle(ctx):
    rng = np.random.default_rng(9)
    good = orc.encode(lzma_amd.bench_generate(20000).tobytes(), orc.params(dict_size=1 << 16, fb=32))
    streams = []
    for k in range(40):
        b = bytearray(good)
        for _ in range(3):
            b[int(rng.integers(5, len(b)))] ^= int(rng.integers(1, 256))
        streams.append(bytes(b[: int(rng.integers(5, len(b)))]))
    props = orc.props(orc.params(dict_size=1 << 16, fb=32))
    res = ctx.decode_batch(streams, props, [20000] * len(streams), caps=[20000 + 300] * len(streams))
    for s, (st, d) in zip(streams, res):
        rc, od = orc.decode(s, props, 20000, cap=20000 + 300)
        exp = {1: lzma_amd.LZMA_OK, 0: lzma_amd.LZMA_E_DATA, -1: lzma_amd.LZMA_E_OVERFLOW}[rc]
        assert st == exp
        assert d == od


def test_gpu_decoder_until_end_marker(ctx):
    data = lzma_amd.bench_generate(50000).tobytes()
    p = lzma_amd.make_params(dict_size=1 << 16, fb=32, eos=True)
    blob = lzma_amd.compress_file_bytes(data, p, ctx)
    assert blob == orc.lzma_file(data, _oparams(p))
    assert lzma_amd.decompress_file_bytes(blob, ctx) == data


def test_gpu_java_style_api(ctx):
    """Encoder/Decoder mirrors used exactly like LzmaAlone.java:190-239."""
    data = lzma_amd.bench_generate(30000).tobytes()
    enc = lzma_amd.Encoder(ctx)
    assert enc.SetDictionarySize(1 << 20) and enc.SetNumFastBytes(64) and enc.SetMatchFinder(1)
    assert enc.SetLcLpPb(3, 0, 2)
    enc.SetEndMarkerMode(False)
    out = io.BytesIO()
    enc.WriteCoderProperties(out)
    out.write(len(data).to_bytes(8, "little"))
    enc.Code(io.BytesIO(data), out, -1, -1, None)
    blob = out.getvalue()
    assert blob == orc.lzma_file(data, orc.params(dict_size=1 << 20, fb=64))
    dec = lzma_amd.Decoder(ctx)
    assert dec.SetDecoderProperties(blob[:5])
    res = io.BytesIO()
    assert dec.Code(io.BytesIO(blob[13:]), res, len(data))
    assert res.getvalue() == data


def test_gpu_device_resident_api(ctx):
    torch = pytest.importorskip("torch")
    data = lzma_amd.bench_generate(1 << 20)
    n = 16
    offs = np.linspace(0, data.size, n + 1).astype(np.uint64)
    d_in = torch.from_numpy(data).cuda()
    caps = [lzma_amd.enc_bound(int(offs[i + 1] - offs[i])) for i in range(n)]
    oo = np.zeros(n + 1, dtype=np.uint64)
    oo[1:] = np.cumsum(caps)
    d_out = torch.empty(int(oo[-1]), dtype=torch.uint8, device="cuda")
    p = lzma_amd.make_params(dict_size=1 << 26, fb=32)
    st = torch.cuda.current_stream().cuda_stream
    lens = ctx.encode_batch_dev(d_in, offs, p, d_out, oo, st)
    host_out = d_out.cpu().numpy()
    for i in range(0, n, 5):
        got = host_out[int(oo[i]):int(oo[i] + lens[i])].tobytes()
        assert got == orc.encode(data[int(offs[i]):int(offs[i + 1])].tobytes(), _oparams(p))
    # decode back on device
    d_dec = torch.empty(int(offs[-1]), dtype=torch.uint8, device="cuda")
    in_offs = np.zeros(n + 1, dtype=np.uint64)
    in_offs[1:] = np.cumsum(lens)
    packed = torch.cat([d_out[int(oo[i]):int(oo[i] + lens[i])] for i in range(n)])
    dlens, dst = ctx.decode_batch_dev(lzma_amd.write_props(p), packed, in_offs,
                                      (offs[1:] - offs[:-1]).astype(np.int64), d_dec, offs, st)
    assert (dst == 0).all()
    assert torch.equal(d_dec.cpu(), torch.from_numpy(data))
