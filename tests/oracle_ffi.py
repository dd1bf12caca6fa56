"""ctypes loader for the CPU restatement in oracle/ (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may use
this module; the product library never links the oracle.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "build", "liblzma_oracle.so")


class Params(ctypes.Structure):
    _fields_ = [("dict_size", ctypes.c_int32), ("fb", ctypes.c_int32), ("mf", ctypes.c_int32),
                ("lc", ctypes.c_int32), ("lp", ctypes.c_int32), ("pb", ctypes.c_int32),
                ("eos", ctypes.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        src = os.path.join(ORACLE_DIR, "lzma_oracle.c")
        if not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
        L = ctypes.CDLL(ORACLE_SO)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_encode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(Params), ctypes.c_int,
                                    ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_encode.restype = ctypes.c_int
        L.oracle_free.argtypes = [ctypes.c_void_p]
        L.oracle_decode.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int64,
                                    ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_decode.restype = ctypes.c_int
        L.oracle_write_props.argtypes = [ctypes.POINTER(Params), ctypes.c_void_p]
        L.oracle_match_lists.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(Params),
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64]
        L.oracle_match_lists.restype = ctypes.c_int64
        L.oracle_rc_encode_bits.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
        L.oracle_rc_direct_bits.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                            ctypes.c_int]
        L.oracle_bittree_prices_after.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_enc_new.argtypes = [ctypes.POINTER(Params)]
        L.oracle_enc_new.restype = ctypes.c_void_p
        L.oracle_enc_code.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                      ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_uint64)]
        L.oracle_enc_code.restype = ctypes.c_int
        L.oracle_enc_delete.argtypes = [ctypes.c_void_p]
        L.oracle_prob_price.argtypes = [ctypes.c_int]
        L.oracle_prob_price.restype = ctypes.c_uint32
        _lib = L
    return _lib


def params(dict_size=1 << 23, fb=128, mf=1, lc=3, lp=0, pb=2, eos=0):
    return Params(dict_size, fb, mf, lc, lp, pb, eos)


def _buf(data):
    a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a, a.ctypes.data


def encode(data, p=None, mode=0):
    """Raw stream bytes exactly as Encoder.Code (Encoder.java:1064)."""
    p = p or params()
    a, ptr = _buf(data)
    out = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_uint64()
    rc = lib().oracle_encode(ptr, a.size, ctypes.byref(p), mode, ctypes.byref(out), ctypes.byref(n))
    if rc != 0:
        raise RuntimeError("oracle_encode failed %d" % rc)
    res = ctypes.string_at(out, n.value)
    lib().oracle_free(out)
    return res


class EncoderSession:
    """One reused Encoder instance (oracle_enc_*): match-finder arrays kept
    across calls, hash heads cleared per call as BinTree.Init does
    (BinTree.java:72-80). Not thread-safe: one session per thread."""

    def __init__(self, p):
        self._p = p
        self._h = lib().oracle_enc_new(ctypes.byref(p))
        if not self._h:
            raise RuntimeError("oracle_enc_new failed")

    def encode(self, data):
        a, ptr = _buf(data)
        out = ctypes.POINTER(ctypes.c_uint8)()
        n = ctypes.c_uint64()
        rc = lib().oracle_enc_code(self._h, ptr, a.size, ctypes.byref(out), ctypes.byref(n))
        if rc != 0:
            raise RuntimeError("oracle_enc_code failed %d" % rc)
        return ctypes.string_at(out, n.value)

    def close(self):
        if self._h:
            lib().oracle_enc_delete(self._h)
            self._h = None

    def __del__(self):
        self.close()


def props(p):
    b = (ctypes.c_uint8 * 5)()
    lib().oracle_write_props(ctypes.byref(p), b)
    return bytes(b)


def lzma_file(data, p):
    """.lzma container as LzmaAlone writes it (LzmaAlone.java:208-218)."""
    size = -1 if p.eos else len(data)
    return props(p) + (size & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little") + encode(data, p)


def decode(stream, prop5, out_size, cap=None):
    """Decoder.Code (Decoder.java:205-301). Returns (status, bytes)."""
    cap = cap if cap is not None else (out_size + 64 if out_size >= 0 else len(stream) * 64 + 4096)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    a, ptr = _buf(stream)
    pr = (ctypes.c_uint8 * 5)(*prop5)
    n = ctypes.c_uint64()
    rc = lib().oracle_decode(ptr, a.size, pr, out_size, out.ctypes.data, cap, ctypes.byref(n))
    return rc, out[:n.value].tobytes()


def match_lists(data, p):
    """Per-position (count, main_len, pairs) from BinTree.fillMatches at every position."""
    a, ptr = _buf(data)
    n = a.size
    counts = np.zeros(max(n, 1), dtype=np.uint32)
    main = np.zeros(max(n, 1), dtype=np.uint32)
    cap = n * 8 + 64
    while True:
        lens = np.zeros(cap, dtype=np.uint32)
        dists = np.zeros(cap, dtype=np.uint32)
        tot = lib().oracle_match_lists(ptr, n, ctypes.byref(p), counts.ctypes.data, main.ctypes.data,
                                       lens.ctypes.data, dists.ctypes.data, cap)
        if tot >= 0:
            return counts[:n], main[:n], lens[:tot], dists[:tot]
        cap *= 4


def cpu_threads():
    """Host threads for the oracle: the job's CPU share (OMP_NUM_THREADS on the GPU
    box, else the affinity mask), at most 16."""
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() else len(os.sched_getaffinity(0))
    return max(1, min(n, 16))


def encode_many(chunks, p, threads=None):
    """Oracle encodings of independent chunks on a thread pool, one reused
    EncoderSession per thread (ctypes releases the GIL inside the C calls)."""
    import threading
    from concurrent.futures import ThreadPoolExecutor
    tl = threading.local()
    sessions = []

    def enc(c):
        s = getattr(tl, "s", None)
        if s is None:
            s = tl.s = EncoderSession(p)
            sessions.append(s)
        return s.encode(c)

    with ThreadPoolExecutor(max_workers=threads or cpu_threads()) as ex:
        out = list(ex.map(enc, chunks))
    for s in sessions:
        s.close()
    return out
