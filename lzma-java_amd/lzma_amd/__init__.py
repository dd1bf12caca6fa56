"""lzma_amd -- MI355X-native drop-in for the rfalke/lzma-java LZMA hot path.

Host-side mirror of the reference's codec API, over the C ABI in
include/lzma_mi355x.h (built as lzma-java_amd/build/liblzma_mi355x.so):

  Encoder   <- SevenZip.Compression.LZMA.Encoder  (Encoder.java:16)
  Decoder   <- SevenZip.Compression.LZMA.Decoder  (Decoder.java:12)

Same method names, argument meaning and error behaviour as the Java classes:
setters return False on out-of-range values, Encoder.Code writes the raw
range-coder stream (the caller writes the .lzma header, LzmaAlone.java:
208-217), Decoder.Code returns False on corrupt data. All coding runs on the
GPU; there is no CPU fallback -- without the built library or a HIP device
every coding call raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
# LZMA_AMD_LIB overrides the library path (e.g. the LZG_PROF profiling build)
LIB_PATH = os.environ.get("LZMA_AMD_LIB") or os.path.join(_PKG, "build", "liblzma_mi355x.so")

LZMA_OK = 0
LZMA_E_PARAM = -1
LZMA_E_NOMEM = -2
LZMA_E_DEVICE = -3
LZMA_E_OVERFLOW = -4
LZMA_E_DATA = -5
LZMA_E_NODEVICE = -6
LZMA_E_INTERNAL = -7

EXPORTED_SYMBOLS = [
    "lzma_version", "lzma_params_default", "lzma_params_check", "lzma_write_props", "lzma_read_props",
    "lzma_enc_bound", "lzma_ctx_create", "lzma_ctx_destroy", "lzma_last_error", "lzma_ctx_set_batch_bytes",
    "lzma_ctx_set_timing", "lzma_ctx_timings", "lzma_ctx_reset_timings", "lzma_ctx_stats", "lzma_enc_batch_dev", "lzma_enc_batch",
    "lzma_pack_dev",
    "lzma_encode", "lzma_dec_batch_dev", "lzma_dec_batch", "lzma_decode", "lzma_bench_generate",
    "lzma_rnd_generate", "lzma_text_generate", "lzma_match_lists",
    "lzma_mctx_create", "lzma_mctx_destroy", "lzma_mctx_last_error", "lzma_mctx_devices",
    "lzma_enc_batch_multi", "lzma_dec_batch_multi", "lzma_mctx_set_batch_bytes", "lzma_mctx_set_timing",
    "lzma_visible_on_error", "lzma_dec_batch_dev_async", "lzma_dec_batch_dev_wait", "lzma_ctx_set_parse_fence",
    "lzma_enc_stage_dev", "lzma_enc_parse_dev_async", "lzma_enc_parse_dev_wait",
    "lzma_enc_session_begin", "lzma_enc_session_step", "lzma_enc_session_save", "lzma_enc_session_restore",
    "lzma_enc_session_end", "lzma_enc_session_begin_host", "lzma_enc_session_output",
]


class LzmaError(RuntimeError):
    def __init__(self, code, msg=""):
        super().__init__("lzma error %d: %s" % (code, msg))
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [("dict_size", ctypes.c_int32), ("fb", ctypes.c_int32), ("mf", ctypes.c_int32),
                ("lc", ctypes.c_int32), ("lp", ctypes.c_int32), ("pb", ctypes.c_int32), ("eos", ctypes.c_int32)]

    def __repr__(self):
        return "Params(dict_size=%d, fb=%d, mf=%d, lc=%d, lp=%d, pb=%d, eos=%d)" % (
            self.dict_size, self.fb, self.mf, self.lc, self.lp, self.pb, self.eos)


_lib_handle = None


def lib():
    """Load the product library; raises if it was not built (no fallback)."""
    global _lib_handle
    if _lib_handle is None:
        if not os.path.exists(LIB_PATH):
            raise LzmaError(LZMA_E_INTERNAL, "%s not built (run `make -C lzma-java_amd` or "
                                             "__graft_entry__.build())" % LIB_PATH)
        # PyTorch-ROCm wheels bundle their own libamdhip64 (SONAME
        # libamdhip64.so.7). Load it first so our DT_NEEDED resolves to the same
        # runtime: one HIP/HSA instance per process, and torch's hipStream_t
        # handles are valid streams for the device-resident entry points.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
        P = ctypes.POINTER(Params)
        L.lzma_version.restype = ctypes.c_char_p
        L.lzma_params_default.argtypes = [P]
        L.lzma_params_check.argtypes = [P]
        L.lzma_write_props.argtypes = [P, vp]
        L.lzma_read_props.argtypes = [vp, P]
        L.lzma_enc_bound.argtypes = [u64]
        L.lzma_enc_bound.restype = u64
        L.lzma_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
        L.lzma_ctx_destroy.argtypes = [vp]
        L.lzma_last_error.argtypes = [vp]
        L.lzma_last_error.restype = ctypes.c_char_p
        L.lzma_ctx_set_batch_bytes.argtypes = [vp, u64]
        L.lzma_ctx_set_timing.argtypes = [vp, i32]
        L.lzma_ctx_timings.argtypes = [vp, vp, vp, vp, i32]
        L.lzma_ctx_reset_timings.argtypes = [vp]
        L.lzma_ctx_stats.argtypes = [vp, vp, vp, vp]
        L.lzma_enc_session_begin.argtypes = [vp, P, vp, u64, vp, u64, vp, ctypes.POINTER(vp)]
        L.lzma_enc_session_step.argtypes = [vp, u64, vp, vp, vp]
        L.lzma_enc_session_save.argtypes = [vp, vp, u64, vp]
        L.lzma_enc_session_restore.argtypes = [vp, vp, u64]
        L.lzma_enc_session_end.argtypes = [vp]
        L.lzma_enc_session_begin_host.argtypes = [vp, P, vp, u64, ctypes.POINTER(vp)]
        L.lzma_enc_session_output.argtypes = [vp, u64, vp, u64]
        L.lzma_enc_batch_dev.argtypes = [vp, P, vp, vp, i32, vp, vp, vp, vp]
        L.lzma_enc_batch.argtypes = [vp, P, vp, vp, i32, vp, u64, vp]
        L.lzma_pack_dev.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp]
        L.lzma_encode.argtypes = [vp, P, vp, u64, vp, u64, ctypes.POINTER(u64)]
        L.lzma_dec_batch_dev.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp, vp, vp]
        L.lzma_dec_batch.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp, vp]
        L.lzma_dec_batch_dev_async.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp]
        L.lzma_dec_batch_dev_wait.argtypes = [vp, vp, vp]
        L.lzma_ctx_set_parse_fence.argtypes = [vp, vp]
        L.lzma_enc_stage_dev.argtypes = [vp, P, vp, vp, i32, vp, vp, vp]
        L.lzma_enc_parse_dev_async.argtypes = [vp, vp]
        L.lzma_enc_parse_dev_wait.argtypes = [vp, vp]
        L.lzma_decode.argtypes = [vp, vp, vp, u64, ctypes.c_int64, vp, u64, ctypes.POINTER(u64)]
        L.lzma_bench_generate.argtypes = [vp, u64]
        L.lzma_bench_generate.restype = None
        L.lzma_mctx_create.argtypes = [ctypes.c_uint32, ctypes.POINTER(vp)]
        L.lzma_mctx_destroy.argtypes = [vp]
        L.lzma_mctx_last_error.argtypes = [vp]
        L.lzma_mctx_last_error.restype = ctypes.c_char_p
        L.lzma_mctx_devices.argtypes = [vp]
        L.lzma_mctx_set_batch_bytes.argtypes = [vp, u64]
        L.lzma_mctx_set_timing.argtypes = [vp, i32]
        L.lzma_visible_on_error.argtypes = [ctypes.c_uint32, u64]
        L.lzma_visible_on_error.restype = u64
        L.lzma_enc_batch_multi.argtypes = [vp, P, vp, vp, i32, vp, u64, vp]
        L.lzma_dec_batch_multi.argtypes = [vp, vp, vp, vp, i32, vp, vp, vp, vp, vp]
        L.lzma_match_lists.argtypes = [vp, P, vp, vp, i32, vp, vp, vp, vp, u64, ctypes.POINTER(u64)]
        L.lzma_rnd_generate.argtypes = [vp, u64, u64]
        L.lzma_rnd_generate.restype = None
        L.lzma_text_generate.argtypes = [vp, u64, u64]
        L.lzma_text_generate.restype = None
        _lib_handle = L
    return _lib_handle


def version() -> str:
    return lib().lzma_version().decode()


def default_params() -> Params:
    p = Params()
    lib().lzma_params_default(ctypes.byref(p))
    return p


def make_params(dict_size=1 << 22, fb=32, mf=1, lc=3, lp=0, pb=2, eos=False) -> Params:
    return Params(int(dict_size), int(fb), int(mf), int(lc), int(lp), int(pb), 1 if eos else 0)


def params_ok(p: Params) -> bool:
    return lib().lzma_params_check(ctypes.byref(p)) == LZMA_OK


def write_props(p: Params) -> bytes:
    b = (ctypes.c_uint8 * 5)()
    lib().lzma_write_props(ctypes.byref(p), b)
    return bytes(b)


def read_props(props: bytes) -> Optional[Params]:
    p = Params()
    b = (ctypes.c_uint8 * 5)(*props[:5])
    return p if lib().lzma_read_props(b, ctypes.byref(p)) == LZMA_OK else None


def enc_bound(n: int) -> int:
    return int(lib().lzma_enc_bound(n))


def visible_on_error(dict_size: int, decoded_len: int) -> int:
    """Bytes Decoder.Code has written when it returns false after decoding
    decoded_len bytes: the whole windows OutWindow flushed (lzma_visible_on_error)."""
    return int(lib().lzma_visible_on_error(dict_size & 0xFFFFFFFF, decoded_len))


def bench_generate(size: int) -> np.ndarray:
    """LzmaBench.CBenchRandomGenerator output (LzmaBench.java:104-127)."""
    buf = np.empty(max(size, 1), dtype=np.uint8)
    lib().lzma_bench_generate(buf.ctypes.data, size)
    return buf[:size]


def rnd_generate(size: int, seed: int = 0x5EED) -> np.ndarray:
    """RND input of SURVEY.md 8(d): SplitMix64 bytes (config 1: 1 MiB, seed 0x5EED)."""
    buf = np.empty(max(size, 1), dtype=np.uint8)
    lib().lzma_rnd_generate(buf.ctypes.data, size, seed)
    return buf[:size]


def text_generate(size: int, seed: int = 1) -> np.ndarray:
    """TEXT ("enwik9-shaped") input of SURVEY.md 8(d): Zipf(1.1) words, wiki markup (config 3: seed 1)."""
    buf = np.empty(max(size, 1), dtype=np.uint8)
    lib().lzma_text_generate(buf.ctypes.data, size, seed)
    return buf[:size]


def generate(kind: str, size: int) -> np.ndarray:
    """Synthetic input by name: 'bench' (LzmaBench), 'text' (config 3) or 'rnd' (config 1)."""
    if kind == "bench":
        return bench_generate(size)
    if kind == "text":
        return text_generate(size)
    if kind == "rnd":
        return rnd_generate(size)
    raise ValueError("unknown input kind %r" % kind)


class Context:
    """One HIP device plus its device workspace (lzma_ctx)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        rc = lib().lzma_ctx_create(device, ctypes.byref(h))
        if rc != LZMA_OK:
            raise LzmaError(rc, "lzma_ctx_create(device=%d) failed%s" % (
                device, " (no HIP device; the MI355X path has no CPU fallback)" if rc == LZMA_E_NODEVICE else ""))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib().lzma_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self) -> str:
        return lib().lzma_last_error(self.h).decode()

    def check(self, rc):
        if rc != LZMA_OK:
            raise LzmaError(rc, self.error())

    def set_batch_bytes(self, n: int):
        self.check(lib().lzma_ctx_set_batch_bytes(self.h, n))

    def set_timing(self, on: bool):
        self.check(lib().lzma_ctx_set_timing(self.h, 1 if on else 0))

    def timings(self) -> dict:
        cap = 32
        names = (ctypes.c_char_p * cap)()
        ms = (ctypes.c_double * cap)()
        n = (ctypes.c_int64 * cap)()
        k = lib().lzma_ctx_timings(self.h, names, ms, n, cap)
        return {names[i].decode(): (ms[i], n[i]) for i in range(k)}

    def reset_timings(self):
        lib().lzma_ctx_reset_timings(self.h)

    def stats(self) -> dict:
        """lzma_ctx_stats: cumulative allocations (count, bytes) and whole-device syncs."""
        v = (ctypes.c_uint64 * 3)()
        self.check(lib().lzma_ctx_stats(self.h, ctypes.byref(v, 0), ctypes.byref(v, 8), ctypes.byref(v, 16)))
        return {"allocations": int(v[0]), "alloc_bytes": int(v[1]), "device_syncs": int(v[2])}

    # ---- host-buffer batch API
    def encode_batch(self, streams: Sequence[bytes], p: Params) -> List[bytes]:
        arrs = [np.frombuffer(s, dtype=np.uint8) if not isinstance(s, np.ndarray) else s for s in streams]
        offs = np.zeros(len(arrs) + 1, dtype=np.uint64)
        np.cumsum([a.size for a in arrs], out=offs[1:])
        data = np.concatenate(arrs) if arrs and offs[-1] > 0 else np.zeros(1, dtype=np.uint8)
        cap = int(sum(enc_bound(a.size) for a in arrs)) + 1
        out = np.empty(cap, dtype=np.uint8)
        oo = np.zeros(len(arrs) + 1, dtype=np.uint64)
        self.check(lib().lzma_enc_batch(self.h, ctypes.byref(p), data.ctypes.data, offs.ctypes.data, len(arrs),
                                        out.ctypes.data, cap, oo.ctypes.data))
        return [out[oo[i]:oo[i + 1]].tobytes() for i in range(len(arrs))]

    def decode_batch(self, streams: Sequence[bytes], props: bytes, out_sizes: Sequence[int],
                     caps: Optional[Sequence[int]] = None) -> List[Tuple[int, bytes]]:
        arrs = [np.frombuffer(s, dtype=np.uint8) for s in streams]
        n = len(arrs)
        io = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum([a.size for a in arrs], out=io[1:])
        data = np.concatenate(arrs) if n and io[-1] > 0 else np.zeros(1, dtype=np.uint8)
        if caps is None:
            caps = [s if s >= 0 else max(64 * a.size, 4096) for s, a in zip(out_sizes, arrs)]
        oo = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(caps, out=oo[1:])
        out = np.zeros(int(oo[-1]) + 1, dtype=np.uint8)
        sizes = np.array(out_sizes, dtype=np.int64)
        lens = np.zeros(n, dtype=np.uint64)
        status = np.zeros(n, dtype=np.int32)
        self.check(lib().lzma_dec_batch(self.h, (ctypes.c_uint8 * 5)(*props[:5]), data.ctypes.data, io.ctypes.data, n,
                                        sizes.ctypes.data, out.ctypes.data, oo.ctypes.data, lens.ctypes.data,
                                        status.ctypes.data))
        res = []
        for i in range(n):
            L = min(int(lens[i]), int(oo[i + 1] - oo[i]))
            res.append((int(status[i]), out[oo[i]:oo[i] + L].tobytes()))
        return res

    def match_lists(self, streams: Sequence[bytes], p: Params):
        """The GPU match finder's output (lzma_match_lists): per input byte of the
        concatenated streams (count, main_len), and all pairs in position order."""
        arrs = [np.frombuffer(s, dtype=np.uint8) if not isinstance(s, np.ndarray) else s for s in streams]
        offs = np.zeros(len(arrs) + 1, dtype=np.uint64)
        np.cumsum([a.size for a in arrs], out=offs[1:])
        data = np.concatenate(arrs) if arrs and offs[-1] > 0 else np.zeros(1, dtype=np.uint8)
        n = int(offs[-1])
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        main = np.zeros(max(n, 1), dtype=np.uint32)
        cap = max(n * 4, 64)
        while True:
            lens = np.zeros(cap, dtype=np.uint32)
            dists = np.zeros(cap, dtype=np.uint32)
            tot = ctypes.c_uint64()
            rc = lib().lzma_match_lists(self.h, ctypes.byref(p), data.ctypes.data, offs.ctypes.data, len(arrs),
                                        counts.ctypes.data, main.ctypes.data, lens.ctypes.data, dists.ctypes.data,
                                        cap, ctypes.byref(tot))
            if rc == LZMA_E_OVERFLOW:
                cap = int(tot.value)
                continue
            self.check(rc)
            k = int(tot.value)
            return counts[:n], main[:n], lens[:k], dists[:k]

    # ---- device-resident batch API (torch tensors already in HBM)
    def encode_batch_dev(self, d_in, offs: np.ndarray, p: Params, d_out, out_offs: np.ndarray, stream_ptr: int = 0):
        """d_in/d_out: device pointers (int) or torch uint8 cuda tensors."""
        n = len(offs) - 1
        lens = np.zeros(max(n, 1), dtype=np.uint64)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        out_offs = np.ascontiguousarray(out_offs, dtype=np.uint64)
        self.check(lib().lzma_enc_batch_dev(self.h, ctypes.byref(p), _dptr(d_in), offs.ctypes.data, n, _dptr(d_out),
                                            out_offs.ctypes.data, lens.ctypes.data, ctypes.c_void_p(stream_ptr)))
        return lens[:n]

    # the same encode in three calls (lzma_enc_stage_dev / _parse_dev_async / _parse_dev_wait):
    # the range coder of one batch runs on the context's coder stream while the next
    # batch's match finder runs on the caller's stream
    def encode_stage_dev(self, d_in, offs: np.ndarray, p: Params, d_out, out_offs: np.ndarray, stream_ptr: int = 0) -> None:
        """Stage a batch and enqueue its match finder's keys and sorts (at most two batches
        staged: the newer one's walk then runs beside the older one's parse)."""
        n = len(offs) - 1
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        out_offs = np.ascontiguousarray(out_offs, dtype=np.uint64)
        self.check(lib().lzma_enc_stage_dev(self.h, ctypes.byref(p), _dptr(d_in), offs.ctypes.data, n, _dptr(d_out),
                                            out_offs.ctypes.data, ctypes.c_void_p(stream_ptr)))
        self._staged = getattr(self, "_staged", []) + [n]

    def encode_parse_dev_async(self, stream_ptr: int = 0) -> None:
        """The oldest staged batch's walk and parser on the caller's stream, its range coder
        on the context's coder stream; returns without waiting for them."""
        rc = lib().lzma_enc_parse_dev_async(self.h, ctypes.c_void_p(stream_ptr))
        staged = getattr(self, "_staged", [])
        if rc != LZMA_OK:
            if rc != LZMA_E_PARAM:   # a refusal consumes nothing; a failed parse drops every staged batch
                self._staged = []
            self.check(rc)
        self._coders = getattr(self, "_coders", []) + [staged[0] if staged else 0]
        self._staged = staged[1:]

    def encode_parse_dev_wait(self) -> np.ndarray:
        """Wait for the oldest range coder in flight; its batch's encoded lengths."""
        coders = getattr(self, "_coders", [])
        n = coders[0] if coders else 0
        lens = np.zeros(max(n, 1), dtype=np.uint64)
        rc = lib().lzma_enc_parse_dev_wait(self.h, lens.ctypes.data)
        if rc != LZMA_E_PARAM:   # collected (or failed): the oldest coder is gone
            self._coders = coders[1:]
        self.check(rc)
        return lens[:n]

    def pack_dev(self, d_src, src_offs: np.ndarray, lens: np.ndarray, d_dst, stream_ptr: int = 0) -> np.ndarray:
        """Gather capacity-layout streams into a contiguous buffer; returns the packed offsets."""
        n = len(lens)
        src_offs = np.ascontiguousarray(src_offs, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        dst = np.zeros(n + 1, dtype=np.uint64)
        dst[1:] = np.cumsum(lens)
        self.check(lib().lzma_pack_dev(self.h, _dptr(d_src), src_offs.ctypes.data, lens.ctypes.data, n, _dptr(d_dst),
                                       dst.ctypes.data, ctypes.c_void_p(stream_ptr)))
        return dst

    def decode_batch_dev(self, props: bytes, d_in, in_offs: np.ndarray, out_sizes: np.ndarray, d_out,
                         out_offs: np.ndarray, stream_ptr: int = 0):
        n = len(in_offs) - 1
        in_offs = np.ascontiguousarray(in_offs, dtype=np.uint64)
        out_offs = np.ascontiguousarray(out_offs, dtype=np.uint64)
        sizes = np.ascontiguousarray(out_sizes, dtype=np.int64)
        lens = np.zeros(max(n, 1), dtype=np.uint64)
        status = np.zeros(max(n, 1), dtype=np.int32)
        self.check(lib().lzma_dec_batch_dev(self.h, (ctypes.c_uint8 * 5)(*props[:5]), _dptr(d_in), in_offs.ctypes.data,
                                            n, sizes.ctypes.data, _dptr(d_out), out_offs.ctypes.data,
                                            lens.ctypes.data, status.ctypes.data, ctypes.c_void_p(stream_ptr)))
        return lens[:n], status[:n]

    def decode_batch_dev_async(self, props: bytes, d_in, in_offs: np.ndarray, out_sizes: np.ndarray, d_out,
                               out_offs: np.ndarray, stream_ptr: int = 0) -> None:
        """Enqueue a batch decode and return at once; decode_batch_dev_wait() gives (lens, status)."""
        n = len(in_offs) - 1
        in_offs = np.ascontiguousarray(in_offs, dtype=np.uint64)
        out_offs = np.ascontiguousarray(out_offs, dtype=np.uint64)
        sizes = np.ascontiguousarray(out_sizes, dtype=np.int64)
        self.check(lib().lzma_dec_batch_dev_async(self.h, (ctypes.c_uint8 * 5)(*props[:5]), _dptr(d_in),
                                                  in_offs.ctypes.data, n, sizes.ctypes.data, _dptr(d_out),
                                                  out_offs.ctypes.data, ctypes.c_void_p(stream_ptr)))
        self._async_n = n

    def decode_batch_dev_wait(self):
        n = getattr(self, "_async_n", 0)
        lens = np.zeros(max(n, 1), dtype=np.uint64)
        status = np.zeros(max(n, 1), dtype=np.int32)
        self.check(lib().lzma_dec_batch_dev_wait(self.h, lens.ctypes.data, status.ctypes.data))
        self._async_n = 0
        return lens[:n], status[:n]

    def session(self, d_in, n: int, p: Params, d_out, out_cap: int, stream_ptr: int = 0, resume: bytes = None):
        """An EncodeSession (the sliced encode of one stream) on this context."""
        return EncodeSession(self, d_in, n, p, d_out, out_cap, stream_ptr, resume)

    def session_host(self, data: bytes, p: Params):
        """An EncodeSession over host bytes (lzma_enc_session_begin_host); read its output with .output()."""
        return EncodeSession(self, None, len(data), p, None, 0, host=data)

    def set_parse_fence(self, dec_ctx: "Context | None") -> None:
        """Encode passes on this context start their parser only after dec_ctx's
        asynchronous decode in flight has finished (None clears it)."""
        self.check(lib().lzma_ctx_set_parse_fence(self.h, dec_ctx.h if dec_ctx is not None else None))


def blob_positions(blob: bytes):
    """(input consumed, final output bytes, done) recorded in a session blob (runtime.hip B_*)."""
    w = np.frombuffer(blob[:11 * 8], dtype=np.uint64)
    return int(w[8]), int(w[9]), bool(w[10])


class EncodeSession:
    """The sliced encode of ONE stream (lzma_enc_session_*): Encoder.Code (Encoder.java:1064-1077)
    in bounded launches. step(nbytes) parses and codes at least nbytes more input and appends
    the final output bytes; save() / Context.session(..., resume=blob) carry the state to another
    process. d_in / d_out: device pointers or torch tensors, valid until close()."""

    def __init__(self, ctx: "Context", d_in, n: int, p: Params, d_out, out_cap: int, stream_ptr: int = 0,
                 resume: bytes = None, host: bytes = None):
        self.ctx = ctx
        self.h = ctypes.c_void_p()
        if host is not None:   # lzma_enc_session_begin_host: the input from host memory
            self._src = np.frombuffer(host, dtype=np.uint8) if not isinstance(host, np.ndarray) else host
            ctx.check(lib().lzma_enc_session_begin_host(ctx.h, ctypes.byref(p), self._src.ctypes.data, self._src.size,
                                                        ctypes.byref(self.h)))
        else:
            ctx.check(lib().lzma_enc_session_begin(ctx.h, ctypes.byref(p), _dptr(d_in), n, _dptr(d_out), out_cap,
                                                   ctypes.c_void_p(stream_ptr), ctypes.byref(self.h)))
        self.in_pos, self.out_len, self.done = 0, 0, False
        if resume is not None:
            buf = (ctypes.c_uint8 * len(resume)).from_buffer_copy(resume)
            rc = lib().lzma_enc_session_restore(self.h, buf, len(resume))
            if rc != LZMA_OK:
                self.close()
                ctx.check(rc)
            self.in_pos, self.out_len, self.done = blob_positions(resume)

    def step(self, nbytes: int):
        """(input consumed, final output bytes, done) after at least nbytes more input."""
        ip, ol, dn = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        self.ctx.check(lib().lzma_enc_session_step(self.h, nbytes, ctypes.byref(ip), ctypes.byref(ol), ctypes.byref(dn)))
        self.in_pos, self.out_len, self.done = int(ip.value), int(ol.value), bool(dn.value)
        return self.in_pos, self.out_len, self.done

    def output(self, start: int, length: int) -> bytes:
        """lzma_enc_session_output: final output bytes [start, start + length) to the host."""
        buf = np.zeros(max(length, 1), dtype=np.uint8)
        self.ctx.check(lib().lzma_enc_session_output(self.h, start, buf.ctypes.data, length))
        return buf[:length].tobytes()

    def save(self) -> bytes:
        n = ctypes.c_uint64()
        self.ctx.check(lib().lzma_enc_session_save(self.h, None, 0, ctypes.byref(n)))
        buf = (ctypes.c_uint8 * n.value)()
        self.ctx.check(lib().lzma_enc_session_save(self.h, buf, n.value, ctypes.byref(n)))
        return bytes(buf[:n.value])

    def close(self):
        if self.h:
            lib().lzma_enc_session_end(self.h)
            self.h = ctypes.c_void_p()


class MultiContext:
    """Several devices from one process (lzma_mctx, SURVEY 8(b) device_mask):
    the batch calls deal the streams round-robin over the devices in the mask.

    Not a Context subclass: an lzma_mctx handle is not an lzma_ctx, so only the
    operations the multi-device C entry points provide exist here (the C side
    also rejects a handle of the wrong kind with LZMA_E_PARAM)."""

    def __init__(self, device_mask: int):
        h = ctypes.c_void_p()
        rc = lib().lzma_mctx_create(device_mask, ctypes.byref(h))
        if rc != LZMA_OK:
            raise LzmaError(rc, "lzma_mctx_create(mask=0x%x) failed" % device_mask)
        self.h = h
        self.device_mask = device_mask
        self.devices = lib().lzma_mctx_devices(h)

    def close(self):
        if self.h:
            lib().lzma_mctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def error(self) -> str:
        return lib().lzma_mctx_last_error(self.h).decode()

    def check(self, rc):
        if rc != LZMA_OK:
            raise LzmaError(rc, self.error())

    def set_batch_bytes(self, n: int):
        self.check(lib().lzma_mctx_set_batch_bytes(self.h, n))

    def set_timing(self, on: bool):
        self.check(lib().lzma_mctx_set_timing(self.h, 1 if on else 0))

    def encode_batch(self, streams: Sequence[bytes], p: Params) -> List[bytes]:
        arrs = [np.frombuffer(s, dtype=np.uint8) if not isinstance(s, np.ndarray) else s for s in streams]
        offs = np.zeros(len(arrs) + 1, dtype=np.uint64)
        np.cumsum([a.size for a in arrs], out=offs[1:])
        data = np.concatenate(arrs) if arrs and offs[-1] > 0 else np.zeros(1, dtype=np.uint8)
        cap = int(sum(enc_bound(a.size) for a in arrs)) + 1
        out = np.empty(cap, dtype=np.uint8)
        oo = np.zeros(len(arrs) + 1, dtype=np.uint64)
        self.check(lib().lzma_enc_batch_multi(self.h, ctypes.byref(p), data.ctypes.data, offs.ctypes.data, len(arrs),
                                              out.ctypes.data, cap, oo.ctypes.data))
        return [out[oo[i]:oo[i + 1]].tobytes() for i in range(len(arrs))]

    def decode_batch(self, streams: Sequence[bytes], props: bytes, out_sizes: Sequence[int],
                     caps: Optional[Sequence[int]] = None) -> List[Tuple[int, bytes]]:
        arrs = [np.frombuffer(s, dtype=np.uint8) for s in streams]
        n = len(arrs)
        io = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum([a.size for a in arrs], out=io[1:])
        data = np.concatenate(arrs) if n and io[-1] > 0 else np.zeros(1, dtype=np.uint8)
        if caps is None:
            caps = [s if s >= 0 else max(64 * a.size, 4096) for s, a in zip(out_sizes, arrs)]
        oo = np.zeros(n + 1, dtype=np.uint64)
        np.cumsum(caps, out=oo[1:])
        out = np.zeros(int(oo[-1]) + 1, dtype=np.uint8)
        sizes = np.array(out_sizes, dtype=np.int64)
        lens = np.zeros(max(n, 1), dtype=np.uint64)
        status = np.zeros(max(n, 1), dtype=np.int32)
        self.check(lib().lzma_dec_batch_multi(self.h, (ctypes.c_uint8 * 5)(*props[:5]), data.ctypes.data,
                                              io.ctypes.data, n, sizes.ctypes.data, out.ctypes.data, oo.ctypes.data,
                                              lens.ctypes.data, status.ctypes.data))
        return [(int(status[i]), out[oo[i]:oo[i] + min(int(lens[i]), int(oo[i + 1] - oo[i]))].tobytes())
                for i in range(n)]


def _dptr(x) -> ctypes.c_void_p:
    if hasattr(x, "data_ptr"):
        return ctypes.c_void_p(x.data_ptr())
    return ctypes.c_void_p(int(x))


_default_ctx = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(0)
    return _default_ctx


# --------------------------------------------------------------------------
# Drop-in mirrors of the Java classes
# --------------------------------------------------------------------------

def _read_all(stream) -> bytes:
    if isinstance(stream, (bytes, bytearray, memoryview)):
        return bytes(stream)
    chunks = []
    while True:
        b = stream.read(1 << 20)
        if not b:
            break
        chunks.append(b)
    return b"".join(chunks)


class Encoder:
    """Mirror of SevenZip.Compression.LZMA.Encoder (Encoder.java:16-1185)."""

    EMatchFinderTypeBT2 = 0
    EMatchFinderTypeBT4 = 1
    kDefaultDictionaryLogSize = 22
    kNumFastBytesDefault = 0x20

    def __init__(self, ctx: Optional[Context] = None):
        self._ctx = ctx
        self._p = make_params()
        self._p.dict_size = 1 << self.kDefaultDictionaryLogSize
        self._p.fb = self.kNumFastBytesDefault

    @staticmethod
    def SetAlgorithm(algorithm: int) -> bool:   # Encoder.java:1127-1133 (a no-op in the reference)
        return True

    def SetDictionarySize(self, dictionarySize: int) -> bool:   # :1135-1146
        if dictionarySize < 1 or dictionarySize > (1 << 29):
            return False
        self._p.dict_size = dictionarySize
        return True

    def SetNumFastBytes(self, numFastBytes: int) -> bool:   # :1148-1154
        if numFastBytes < 5 or numFastBytes > 273:
            return False
        self._p.fb = numFastBytes
        return True

    def SetMatchFinder(self, matchFinderIndex: int) -> bool:   # :1156-1167
        if matchFinderIndex < 0 or matchFinderIndex > 2:
            return False
        self._p.mf = matchFinderIndex
        return True

    def SetLcLpPb(self, lc: int, lp: int, pb: int) -> bool:   # :1169-1180
        if lp < 0 or lp > 4 or lc < 0 or lc > 8 or pb < 0 or pb > 4:
            return False
        self._p.lc, self._p.lp, self._p.pb = lc, lp, pb
        return True

    def SetEndMarkerMode(self, endMarkerMode: bool):   # :1182-1184
        self._p.eos = 1 if endMarkerMode else 0

    def params(self) -> Params:
        return Params(*[getattr(self._p, f) for f, _ in Params._fields_])

    def WriteCoderProperties(self, outStream):   # :1079-1085
        outStream.write(write_props(self._p))

    # input bytes per device launch of a long stream's sliced encode (lzma_enc_session_*)
    SLICE_BYTES = 16 << 20

    def Code(self, inStream, outStream, inSize: int = -1, outSize: int = -1, progress=None):   # :1064-1077
        data = _read_all(inStream)
        ctx = self._ctx or default_context()
        if len(data) > self.SLICE_BYTES:
            # slice by slice (the same bytes): each slice's final output is written as it is
            # produced and progress reported per slice, as the reference writes while it codes
            # and reports per block (Encoder.java:1069-1073)
            s = ctx.session_host(data, self._p)
            try:
                written = 0
                while not s.done:
                    in_pos, out_len, _ = s.step(self.SLICE_BYTES)
                    outStream.write(s.output(written, out_len - written))
                    written = out_len
                    if progress is not None:
                        progress.SetProgress(in_pos, out_len)
            finally:
                s.close()
            return
        out = ctx.encode_batch([data], self._p)[0]
        outStream.write(out)
        if progress is not None:   # ICodeProgress.SetProgress, once at the end (no output bits depend on it)
            progress.SetProgress(len(data), len(out))


class Decoder:
    """Mirror of SevenZip.Compression.LZMA.Decoder (Decoder.java:12-319)."""

    def __init__(self, ctx: Optional[Context] = None):
        self._ctx = ctx
        self._props = None

    def SetDecoderProperties(self, properties: bytes) -> bool:   # :303-318
        if len(properties) < 5:
            return False
        if read_props(bytes(properties[:5])) is None:
            return False
        self._props = bytes(properties[:5])
        return True

    def Code(self, inStream, outStream, outSize: int) -> bool:   # :205-301
        if self._props is None:
            raise LzmaError(LZMA_E_PARAM, "SetDecoderProperties first")
        data = _read_all(inStream)
        ctx = self._ctx or default_context()
        cap = outSize if outSize >= 0 else max(64 * len(data), 1 << 16)
        while True:
            # the loop of Decoder.java:219 stops at outSize only between symbols: a final
            # match may run up to kMatchMaxLen (273) bytes past it and is written whole
            st, out = ctx.decode_batch([data], self._props, [outSize], caps=[cap + 273])[0]
            if st == LZMA_E_OVERFLOW and outSize < 0:
                cap *= 4
                continue
            break
        if st not in (LZMA_OK, LZMA_E_DATA):
            # not a verdict on the data (the reference throws, as the JNI shim does): no
            # unvalidated output reaches the caller's stream
            raise LzmaError(st, "Decoder.Code: status %d" % st)
        if st == LZMA_E_DATA:
            # Code returns false with only the whole windows OutWindow flushed so far
            # written (OutWindow.java:63-73; window = max(dict, 4096), Decoder.java:167)
            dict_size = int.from_bytes(self._props[1:5], "little")
            out = out[:visible_on_error(dict_size, len(out))]
        outStream.write(out)
        return st == LZMA_OK


# --------------------------------------------------------------------------
# .lzma container (LzmaAlone.java:208-236) and multi-stream framing
# --------------------------------------------------------------------------

def lzma_header(p: Params, size: int) -> bytes:
    """5 property bytes + 8-byte little-endian size (-1 with the end marker)."""
    return write_props(p) + (size & 0xFFFFFFFFFFFFFFFF).to_bytes(8, "little")


def compress_file_bytes(data: bytes, p: Params, ctx: Optional[Context] = None) -> bytes:
    """LzmaAlone `e`: header + Encoder.Code output."""
    ctx = ctx or default_context()
    return lzma_header(p, -1 if p.eos else len(data)) + ctx.encode_batch([data], p)[0]


def decompress_file_bytes(blob: bytes, ctx: Optional[Context] = None) -> bytes:
    """LzmaAlone `d`: parse header, Decoder.Code; raises on corrupt data."""
    if len(blob) < 13:
        raise LzmaError(LZMA_E_DATA, "input .lzma file is too short")
    d = Decoder(ctx)
    if not d.SetDecoderProperties(blob[:5]):
        raise LzmaError(LZMA_E_PARAM, "Incorrect stream properties")
    size = int.from_bytes(blob[5:13], "little", signed=True)
    import io
    out = io.BytesIO()
    if not d.Code(blob[13:], out, size):
        raise LzmaError(LZMA_E_DATA, "Error in data stream")
    return out.getvalue()
