"""The pipelined batch API (lzma_dec_batch_dev_async / _wait and
lzma_ctx_set_parse_fence, include/lzma_mi355x.h) through the product sources
compiled for the CPU SIMT emulation (tests/simt): the async decode's outputs
equal the synchronous decode's and the oracle's input bytes, a context with a
decode in flight refuses other work, and the fence checks its handles.
Host logic only; the GPU schedule itself is measured by bench.py --overlap."""
import multiprocessing as mp
import os
import subprocess

import numpy as np
import pytest

SIMT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "simt")
SIMT_LIB = os.path.join(SIMT, "build", "so", "libsimt_lzma.so")


def _worker(q):
    import lzma_amd
    lzma_amd.LIB_PATH = SIMT_LIB   # "device" pointers are host pointers in the emulation
    try:
        data = lzma_amd.bench_generate(5 * 4000 - 777).tobytes()
        streams = [data[i:i + 4000] for i in range(0, len(data), 4000)]
        p = lzma_amd.make_params(dict_size=1 << 20, fb=32)
        props = lzma_amd.write_props(p)
        enc, dec = lzma_amd.Context(0), lzma_amd.Context(0)
        outs = enc.encode_batch(streams, p)
        comp = np.frombuffer(b"".join(outs) + b"\0", dtype=np.uint8).copy()
        in_offs = np.zeros(len(outs) + 1, dtype=np.uint64)
        in_offs[1:] = np.cumsum([len(o) for o in outs])
        sizes = np.array([len(s) for s in streams], dtype=np.int64)
        out_offs = np.zeros(len(streams) + 1, dtype=np.uint64)
        out_offs[1:] = np.cumsum(sizes)
        out = np.zeros(int(out_offs[-1]) + 1, dtype=np.uint8)
        enc.set_parse_fence(dec)
        dec.decode_batch_dev_async(props, comp.ctypes.data, in_offs, sizes, out.ctypes.data, out_offs)
        refused = []
        for call in (lambda: dec.decode_batch_dev(props, comp.ctypes.data, in_offs, sizes, out.ctypes.data, out_offs),
                     lambda: dec.decode_batch_dev_async(props, comp.ctypes.data, in_offs, sizes, out.ctypes.data,
                                                        out_offs)):
            try:
                call()
                refused.append(False)
            except lzma_amd.LzmaError as e:
                refused.append(e.code == lzma_amd.LZMA_E_PARAM)
        # an encode on the fenced context while the decode is in flight: allowed (it waits on the device)
        outs2 = enc.encode_batch(streams[:2], p)
        lens, status = dec.decode_batch_dev_wait()
        again = dec.decode_batch_dev_wait()   # nothing in flight: empty, no error
        fence_errs = []
        for bad in (enc, ):   # a context cannot fence on itself
            try:
                enc.set_parse_fence(bad)
                fence_errs.append(False)
            except lzma_amd.LzmaError:
                fence_errs.append(True)
        enc.set_parse_fence(None)
        enc.close()
        dec.close()
        q.put(dict(ok_bytes=out[:int(out_offs[-1])].tobytes() == data, lens=lens.tolist(), status=status.tolist(),
                   sizes=sizes.tolist(), refused=refused, outs2=outs2 == outs[:2], again=len(again[0]),
                   fence_errs=fence_errs))
    except BaseException as e:   # reported to the parent
        q.put(dict(error=repr(e)))


@pytest.mark.timeout(600)
def test_async_decode_and_parse_fence_emulated():
    subprocess.check_call(["make", "-s", "-j", "8", "-C", SIMT, "so"])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    pr = ctx.Process(target=_worker, args=(q,))
    pr.start()
    r = q.get(timeout=500)
    pr.join(timeout=60)
    assert "error" not in r, r.get("error")
    assert r["ok_bytes"]
    assert r["lens"] == r["sizes"] and r["status"] == [0] * len(r["sizes"])
    assert r["refused"] == [True, True]
    assert r["outs2"]
    assert r["again"] == 0
    assert r["fence_errs"] == [True]
