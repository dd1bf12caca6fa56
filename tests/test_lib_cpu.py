"""CPU-side checks of the product library (no GPU needed): it builds, loads,
exports every symbol include/lzma_mi355x.h declares, its host-side helpers
agree with the oracle, and compute entry points fail loudly without a device."""
import ctypes
import os
import re

import numpy as np
import pytest

import lzma_amd
import oracle_ffi as orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    with open(os.path.join(REPO, "include", "lzma_mi355x.h")) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*[\w \*]+?\b(lzma_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points():
    assert set(_declared_symbols()) == set(lzma_amd.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    L = lzma_amd.lib()
    for name in _declared_symbols():
        assert hasattr(L, name), name


def test_version_mentions_gfx950():
    assert "gfx950" in lzma_amd.version()


@pytest.mark.parametrize("kw", [dict(dict_size=1 << 22), dict(dict_size=1, fb=5, lc=0, lp=4, pb=0),
                                dict(dict_size=1 << 29, fb=273, lc=8, lp=0, pb=4, mf=0)])
def test_props_match_oracle(kw):
    p = lzma_amd.make_params(**kw)
    op = orc.params(**{k: int(v) for k, v in kw.items()})
    assert lzma_amd.write_props(p) == orc.props(op)
    q = lzma_amd.read_props(lzma_amd.write_props(p))
    assert (q.lc, q.lp, q.pb, q.dict_size) == (p.lc, p.lp, p.pb, p.dict_size)


def test_params_check_mirrors_setters():
    ok = lzma_amd.make_params()
    assert lzma_amd.params_ok(ok)
    for bad in [dict(dict_size=0), dict(dict_size=(1 << 29) + 1), dict(fb=4), dict(fb=274), dict(mf=3),
                dict(lc=9), dict(lp=5), dict(pb=5)]:
        assert not lzma_amd.params_ok(lzma_amd.make_params(**bad)), bad


def test_encoder_setters_return_false_like_java():
    e = lzma_amd.Encoder()
    assert e.SetDictionarySize(1) and not e.SetDictionarySize(0) and not e.SetDictionarySize((1 << 29) + 1)
    assert e.SetNumFastBytes(5) and not e.SetNumFastBytes(4) and not e.SetNumFastBytes(274)
    assert e.SetMatchFinder(2) and not e.SetMatchFinder(3) and not e.SetMatchFinder(-1)
    assert e.SetLcLpPb(8, 4, 4) and not e.SetLcLpPb(9, 0, 0) and not e.SetLcLpPb(0, 5, 0)
    assert lzma_amd.Encoder.SetAlgorithm(2)


def test_decoder_props_validation():
    d = lzma_amd.Decoder()
    assert not d.SetDecoderProperties(b"\x5d\x00\x00")          # < 5 bytes
    assert not d.SetDecoderProperties(bytes([225, 0, 0, 0, 0]))  # lc/lp/pb out of range
    assert not d.SetDecoderProperties(bytes([0x5d, 0, 0, 0, 0x80]))  # negative dictionary
    assert d.SetDecoderProperties(bytes([0x5d, 0, 0, 0x80, 0]))


def _bench_generate_py(n):
    """Pure-Python restatement of LzmaBench.CBenchRandomGenerator (LzmaBench.java:15-127)."""
    st = {"A1": 362436069, "A2": 521288629, "V": 0, "N": 0}
    M = 0xFFFFFFFF

    def rnd():
        st["A1"] = (36969 * (st["A1"] & 0xFFFF) + (st["A1"] >> 16)) & M
        st["A2"] = (18000 * (st["A2"] & 0xFFFF) + (st["A2"] >> 16)) & M
        return ((st["A1"] << 16) ^ st["A2"]) & M

    def get(nb):
        if st["N"] > nb:
            r = st["V"] & ((1 << nb) - 1)
            st["V"] >>= nb
            st["N"] -= nb
            return r
        nb -= st["N"]
        r = (st["V"] << nb) & M
        st["V"] = rnd()
        r |= st["V"] & ((1 << nb) - 1)
        st["V"] >>= nb
        st["N"] = 32 - nb
        return r

    buf = bytearray(n)
    pos, rep0 = 0, 1
    while pos < n:
        if get(1) == 0 or pos < 1:
            buf[pos] = get(8) & 0xFF
            pos += 1
        else:
            if get(3) == 0:
                ln = 1 + get(1 + get(2))
            else:
                while True:
                    if get(1) == 0:
                        rep0 = get(get(4))
                    else:
                        hi = get(get(4))
                        rep0 = (hi << 10) | get(10)
                    if rep0 < pos:
                        break
                rep0 += 1
                ln = 2 + get(2 + get(2))
            i = 0
            while i < ln and pos < n:
                buf[pos] = buf[pos - rep0]
                i += 1
                pos += 1
    return bytes(buf)


def test_bench_generator_matches_restatement():
    n = 200000
    assert lzma_amd.bench_generate(n).tobytes() == _bench_generate_py(n)


def test_bench_generator_is_low_entropy():
    data = lzma_amd.bench_generate(1 << 18).tobytes()
    out = orc.encode(data, orc.params(dict_size=1 << 18, fb=32))
    assert 0.25 < len(out) / len(data) < 0.45    # ratio ~0.34


def test_no_device_fails_loudly():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(lzma_amd.LzmaError) as ei:
        lzma_amd.Context(0)
    assert ei.value.code == lzma_amd.LZMA_E_NODEVICE
    with pytest.raises(lzma_amd.LzmaError):
        lzma_amd.Encoder().Code(b"abc", __import__("io").BytesIO())


def _fake_handle(magic):
    buf = ctypes.create_string_buffer(512)
    ctypes.memmove(buf, ctypes.c_uint32(magic).value.to_bytes(4, "little"), 4)
    return buf


def test_handles_of_the_wrong_kind_are_rejected():
    # an lzma_mctx* passed where an lzma_ctx* is expected (and the
    # reverse) must be refused with LZMA_E_PARAM, never written through
    L = lzma_amd.lib()
    mctx_like, ctx_like, junk = _fake_handle(0x584D5A4C), _fake_handle(0x58435A4C), _fake_handle(0)
    for h in (mctx_like, junk):
        assert L.lzma_ctx_set_batch_bytes(h, 1 << 30) == lzma_amd.LZMA_E_PARAM
        assert L.lzma_ctx_set_timing(h, 1) == lzma_amd.LZMA_E_PARAM
        assert L.lzma_ctx_timings(h, None, None, None, 0) == lzma_amd.LZMA_E_PARAM
        assert b"invalid" in L.lzma_last_error(h)
        assert bytes(h.raw[4:64]) == b"\0" * 60   # nothing written
    for h in (ctx_like, junk):
        assert L.lzma_mctx_set_batch_bytes(h, 1 << 30) == lzma_amd.LZMA_E_PARAM
        assert L.lzma_mctx_set_timing(h, 1) == lzma_amd.LZMA_E_PARAM
        assert L.lzma_mctx_devices(h) == 0


def test_multicontext_is_not_a_single_device_context():
    assert not issubclass(lzma_amd.MultiContext, lzma_amd.Context)
    for name in ("encode_batch_dev", "decode_batch_dev", "pack_dev", "match_lists", "timings"):
        assert not hasattr(lzma_amd.MultiContext, name), name
    for name in ("set_batch_bytes", "set_timing", "encode_batch", "decode_batch", "close"):
        assert hasattr(lzma_amd.MultiContext, name), name


@pytest.mark.parametrize("dict_size,n,exp", [(1 << 16, 200000, 196608), (1 << 16, 65535, 0), (1, 10000, 8192),
                                             (0, 4095, 0), (1 << 20, (1 << 20) + 5, 1 << 20)])
def test_visible_on_error_is_whole_windows(dict_size, n, exp):
    # Decoder.Code returning false has written only OutWindow's whole-window flushes
    # (OutWindow.java:63-73), window = max(dict, 4096) (Decoder.java:166-167)
    assert lzma_amd.visible_on_error(dict_size, n) == exp


def test_jni_shim_compiles():
    """Compile check of the JNI shim (jni/lzma_jni.c) against a minimal stand-in
    jni.h (tests/jni_stub/): there is no JDK in this container or on the GPU box,
    so this catches C errors before a maintainer with a JDK builds jni/Makefile.
    It is NOT parity evidence: the shim is never linked or called here."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.check_call([cc, "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-Werror",
                           "-I" + os.path.join(repo, "tests", "jni_stub"), "-I" + os.path.join(repo, "include"),
                           os.path.join(repo, "jni", "lzma_jni.c")])
