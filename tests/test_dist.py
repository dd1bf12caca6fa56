"""Multi-rank gather of compressed streams over gloo, world_size 2,
plus the multi-member container. CPU only: the payloads are stand-in byte
strings (the gather moves bytes; it never looks inside them)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as td  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

from lzma_amd import dist  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_data(rank):
    rng = np.random.default_rng(1000 + rank)
    n = 3 + 2 * rank                         # ragged: ranks hold different stream counts
    lens = rng.integers(0, 5000, size=n).astype(np.int64)
    if rank == 1:
        lens[0] = 0                          # an empty stream
    payload = rng.integers(0, 256, size=int(lens.sum()) + 17, dtype=np.uint8)   # slack past the end
    return lens, payload


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        lens, payload = _rank_data(rank)
        out, all_lens, counts = dist.gather_streams(torch.from_numpy(payload), lens, dst=0)
        if rank == 0:
            q.put((out.numpy().tobytes(), all_lens.tolist(), counts.tolist()))
    finally:
        td.destroy_process_group()


def test_gather_streams_gloo_world2():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    blob, all_lens, counts = got
    exp_payload, exp_lens, exp_counts = b"", [], []
    for r in range(world):
        lens, payload = _rank_data(r)
        exp_payload += payload[:int(lens.sum())].tobytes()
        exp_lens += lens.tolist()
        exp_counts.append(len(lens))
    assert counts == exp_counts
    assert all_lens == exp_lens
    assert blob == exp_payload


def test_container_roundtrip():
    props = bytes([0x5D, 0, 0, 0, 4])
    payloads = [b"", b"\x00\x01\x02", bytes(range(256)) * 3]
    sizes = [0, 7, 1 << 20]
    blob = dist.pack_container(props, payloads, sizes)
    members = dist.unpack_container(blob)
    assert len(members) == 3
    for m, pl, n in zip(members, payloads, sizes):
        assert m[:5] == props
        assert int.from_bytes(m[5:13], "little") == n
        assert m[13:] == pl


def test_container_rejects_garbage():
    with pytest.raises(ValueError):
        dist.unpack_container(b"nope" + bytes(20))
    blob = dist.pack_container(bytes(5), [b"abc"], [3])
    with pytest.raises(ValueError):
        dist.unpack_container(blob[:20])   # member table cut short


# ------------------------------------------------------------------ end to end, product kernels emulated

SIMT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "simt")
SIMT_LIB = os.path.join(SIMT, "build", "so", "libsimt_lzma.so")
_CHUNK, _NSTREAMS = 6000, 11


def _e2e_input():
    import lzma_amd
    return lzma_amd.bench_generate(_CHUNK * _NSTREAMS - 1234).tobytes()   # ragged last stream


def _e2e_worker(rank, world, port, q):
    import lzma_amd
    lzma_amd.LIB_PATH = SIMT_LIB   # the product sources, compiled for the CPU SIMT emulation
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    try:
        data = _e2e_input()
        streams = [data[i:i + _CHUNK] for i in range(0, len(data), _CHUNK)]
        mine = dist.rank_streams(len(streams), rank, world)          # {i : i mod G = r}
        p = lzma_amd.make_params(dict_size=1 << 26, fb=32)
        ctx = lzma_amd.Context(0)
        outs = ctx.encode_batch([streams[i] for i in mine], p)
        ctx.close()
        lens = np.array([len(o) for o in outs], dtype=np.int64)
        payload = torch.from_numpy(np.frombuffer(b"".join(outs) + b"\0", dtype=np.uint8).copy())
        out, all_lens, counts = dist.gather_streams(payload, lens, dst=0)
        if rank == 0:
            order = dist.stream_order(counts, world)
            members = dist.reorder_payloads(out.numpy().tobytes(), all_lens, order)
            blob = dist.pack_container(lzma_amd.write_props(p), members, [len(s) for s in streams])
            q.put(blob)
    finally:
        td.destroy_process_group()


@pytest.mark.timeout(600)
def test_round_robin_encode_gather_world2_emulated_kernels():
    """SURVEY 8(e) end to end on CPU: two gloo ranks each encode the streams
    {i : i mod 2 = r} of one buffer with the product kernels (mf/enc/dec.hip
    compiled for the CPU SIMT emulation), rank 0 gathers them with
    dist.gather_streams and writes the multi-member container; every member
    must equal the oracle's Encoder.Code bytes and decode back with the oracle."""
    import subprocess
    import oracle_ffi as orc
    subprocess.check_call(["make", "-s", "-j", "8", "-C", SIMT, "so"])
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_e2e_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    blob = q.get(timeout=500)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = _e2e_input()
    streams = [data[i:i + _CHUNK] for i in range(0, len(data), _CHUNK)]
    members = dist.unpack_container(blob)
    assert len(members) == len(streams)
    op = orc.params(1 << 26, 32, 1, 3, 0, 2, 0)
    for s, m in zip(streams, members):
        assert m[:5] == orc.props(op) and int.from_bytes(m[5:13], "little") == len(s)
        assert m[13:] == orc.encode(s, op)
        rc, d = orc.decode(m[13:], m[:5], len(s))
        assert rc == 1 and d == s


def test_rank_streams_partition():
    for n in (0, 1, 7, 64):
        for world in (1, 2, 3, 8):
            parts = [dist.rank_streams(n, r, world) for r in range(world)]
            allidx = np.sort(np.concatenate(parts)) if n else np.zeros(0)
            assert np.array_equal(allidx, np.arange(n))
            assert np.array_equal(dist.stream_order([len(x) for x in parts], world), np.concatenate(parts))
