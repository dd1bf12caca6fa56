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
